"""ctypes binding of libhdxhash.so (include/hdxhash.h).

The shared library is built in-tree by hyperdex_amd/csrc/Makefile (see
__graft_entry__.build()).  Loading it never touches the GPU; every compute
entry point needs a gfx950 device and returns HDX_E_DEVICE without one —
there is no CPU fallback in this package.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HDX_LIB_PATH") or os.path.join(_HERE, "libhdxhash.so")

HDX_OK = 0
HDX_E_BADTYPE = 1
HDX_E_BADSIZE = 2
HDX_E_DEVICE = 3
HDX_E_INVALID = 4
HDX_E_NOMEM = 5
HDX_E_BADENC = 6
HDX_MAX_ATTRS = 256

STATUS_NAMES = {
    HDX_OK: "HDX_OK", HDX_E_BADTYPE: "HDX_E_BADTYPE", HDX_E_BADSIZE: "HDX_E_BADSIZE",
    HDX_E_DEVICE: "HDX_E_DEVICE", HDX_E_INVALID: "HDX_E_INVALID", HDX_E_NOMEM: "HDX_E_NOMEM",
    HDX_E_BADENC: "HDX_E_BADENC",
}

# Every symbol include/hdxhash.h declares: (name, restype, argtypes)
_u32, _u64, _i32, _sz = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_size_t
_vp, _cp = ctypes.c_void_p, ctypes.c_char_p


class SynthRule(ctypes.Structure):
    _fields_ = [("type", _u32), ("kind", _u32), ("lo", _u32), ("hi", _u32)]


SIGNATURES = [
    ("hdx_abi_version", _i32, []),
    ("hdx_version", _cp, []),
    ("hdx_init", _i32, [_i32]),
    ("hdx_device_count", _i32, []),
    ("hdx_last_error", _cp, []),
    ("hdx_sync", _i32, [_vp]),
    ("hdx_schema_check", _i32, [_vp, _u32]),
    ("hdx_type_hashable", _i32, [_u32]),
    ("hdx_hash_batch_device", _i32, [_vp, _u32, _vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    ("hdx_hash_encoded_device", _i32, [_vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _vp, _vp,
                                       _vp, _vp]),
    ("hdx_synth_encode_values", _i32, [_vp, _vp, _vp, _u32, _u64, _u64, _vp, _vp, _vp]),
    ("hdx_hash_batch_host", _i32, [_vp, _u32, _vp, _u64, _vp, _vp, _u64, _vp]),
    ("hdx_hash_value", _i32, [_u32, _vp, _sz, _vp]),
    ("hdx_hash_key", _i32, [_vp, _u32, _vp, _sz, _vp]),
    ("hdx_hash_object", _i32, [_vp, _u32, _vp, _sz, _vp, _vp, _vp]),
    ("hdx_region_table_create", _i32, [_u32, _u32, _vp, _vp, _vp, _vp, _vp]),
    ("hdx_region_table_destroy", _i32, [_vp]),
    ("hdx_lookup_region_device", _i32, [_vp, _vp, _u32, _u64, _vp, _vp]),
    ("hdx_hash_encoded_regions_device", _i32, [_vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _vp, _u32,
                                               _vp, _vp, _vp, _vp, _vp]),
    ("hdx_hash_batch_regions_device", _i32, [_vp, _u32, _vp, _vp, _vp, _u64, _vp, _u32, _vp, _vp, _vp, _vp]),
    ("hdx_index_key_size", ctypes.c_size_t, [_u32]),
    ("hdx_index_encode_device", _i32, [_u32, _vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    ("hdx_search_regions", _i32, [_vp, _vp, _u32, _vp, _vp]),
    ("hdx_batcher_create", _i32, [_vp, _u32, _vp, _vp]),
    ("hdx_batcher_destroy", _i32, [_vp]),
    ("hdx_batcher_hash_object", _i32, [_vp, _vp, ctypes.c_size_t, _vp, _vp, _vp, _vp]),
    ("hdx_batcher_get_stats", _i32, [_vp, _vp]),
    ("hdx_alloc_pinned", _i32, [_sz, _vp]),
    ("hdx_free_pinned", _i32, [_vp]),
    ("hdx_synth_lengths", _i32, [ctypes.POINTER(SynthRule), _u32, _u64, _u64, _u64, _vp, _vp]),
    ("hdxdbg_set_kernel_variant", _i32, [_i32]),
    ("hdxdbg_kernel_variant", _i32, []),
    ("hdxdbg_kernel_for", _i32, [_vp, _u32, _u64, ctypes.POINTER(ctypes.c_char_p)]),
    ("hdxdbg_stream_probe", _i32, [_vp, _u64, _vp, _i32, _vp]),
    ("hdx_synth_fill", _i32, [ctypes.POINTER(SynthRule), _u32, _u64, _u64, _u64, _vp, _vp, _vp,
                              _u64, _vp]),
]

_LIB = None


class HdxError(RuntimeError):
    """A non-OK hdx_status, with the library's hdx_last_error() message."""

    def __init__(self, status, message):
        super().__init__("%s: %s" % (STATUS_NAMES.get(status, status), message))
        self.status = status


def lib():
    """Load libhdxhash.so (raises if it was not built: no silent fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("hyperdex_amd: %s missing — run __graft_entry__.build() "
                              "(make -C hyperdex_amd/csrc)" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def check(status):
    if status != HDX_OK:
        msg = lib().hdx_last_error()
        raise HdxError(status, msg.decode() if msg else "")
    return status
