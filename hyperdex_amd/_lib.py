"""ctypes binding of libhdxhash.so (include/hdxhash.h).

The shared library is built in-tree by hyperdex_amd/csrc/Makefile (see
__graft_entry__.build()).  Loading it never touches the GPU.  Every batch
entry point needs a gfx950 device and returns HDX_E_DEVICE without one — no
CPU fallback; the per-object signatures of common/hash.h (hdx_hash_value /
_key / _object) are host-CPU code by design (hdx_cpu.cpp).

libhdxhash_dbg.so (same sources, HDX_DEBUG_BUILD) adds the A/B kernel
selection of include/hdxhash_debug.h; tests and scripts/ reach it through
debug_library(), never the product path.
"""
import contextlib
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HDX_LIB_PATH") or os.path.join(_HERE, "libhdxhash.so")
DEBUG_LIB_PATH = os.environ.get("HDX_DEBUG_LIB_PATH") or os.path.join(_HERE, "libhdxhash_dbg.so")

HDX_OK = 0
HDX_E_BADTYPE = 1
HDX_E_BADSIZE = 2
HDX_E_DEVICE = 3
HDX_E_INVALID = 4
HDX_E_NOMEM = 5
HDX_E_BADENC = 6
HDX_MAX_ATTRS = 65535

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


class Shard(ctypes.Structure):
    """struct hdx_shard (include/hdxhash.h): one device's shard."""
    _fields_ = [("blob", _vp), ("obj_base", _vp), ("attr_len", _vp), ("n", _u64), ("coords", _vp),
                ("status_dev", _vp)]


class RegionShard(ctypes.Structure):
    """struct hdx_region_shard (include/hdxhash.h): one device's shard, region-id form."""
    _fields_ = [("blob", _vp), ("obj_base", _vp), ("attr_len", _vp), ("n", _u64), ("region_ids", _vp),
                ("coords", _vp), ("status_dev", _vp)]


SIGNATURES = [
    ("hdx_abi_version", _i32, []),
    ("hdx_version", _cp, []),
    ("hdx_init", _i32, [_i32]),
    ("hdx_init_mask", _i32, [_u64]),
    ("hdx_shutdown", _i32, []),
    ("hdx_device_set", _i32, [_vp, _i32]),
    ("hdx_shard_ranges", _i32, [_vp, _u32, _u64, _u32, ctypes.c_double, _vp]),
    ("hdx_hash_batch_device_multi", _i32, [_vp, _u32, ctypes.POINTER(Shard), _u32, _i32]),
    ("hdx_hash_batch_regions_device_multi", _i32, [_vp, _u32, ctypes.POINTER(RegionShard), _u32, _vp, _u32,
                                                   _i32]),
    ("hdx_hash_batch_regions_host", _i32, [_vp, _u32, _vp, _u64, _vp, _vp, _u64, _vp, _u32, _vp, _vp]),
    ("hdx_hash_encoded_host", _i32, [_vp, _u32, _vp, _u64, _vp, _vp, _vp, _u64, _vp, _vp, _u64, _vp, _vp]),
    ("hdx_hash_encoded_regions_host", _i32, [_vp, _u32, _vp, _u64, _vp, _vp, _vp, _u64, _vp, _vp, _u64, _vp,
                                             _u32, _vp, _vp, _vp]),
    ("hdx_device_count", _i32, []),
    ("hdx_last_error", _cp, []),
    ("hdx_sync", _i32, [_vp]),
    ("hdx_schema_check", _i32, [_vp, _u32]),
    ("hdx_type_hashable", _i32, [_u32]),
    ("hdx_hash_batch_device", _i32, [_vp, _u32, _vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    ("hdx_hash_encoded_device", _i32, [_vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _vp, _vp,
                                       _vp, _vp]),
    ("hdx_synth_encode_values", _i32, [_vp, _vp, _vp, _u32, _u64, _u64, _vp, _vp, _vp]),
    ("hdx_synth_encode_store", _i32, [_vp, _vp, _vp, _u32, _u64, _u64, _vp, _vp, _vp, _vp, _vp]),
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
    ("hdx_search_regions", _i32, [_vp, _vp, _u32, _vp, _vp, _vp]),
    ("hdx_search_space", _i32, [_vp, _u32, _vp, _u32, _vp, _vp, _vp, _vp, _vp]),
    ("hdx_batcher_create", _i32, [_vp, _u32, _vp, _vp]),
    ("hdx_batcher_destroy", _i32, [_vp]),
    ("hdx_batcher_hash_object", _i32, [_vp, _vp, ctypes.c_size_t, _vp, _vp, _vp, _vp]),
    ("hdx_batcher_get_stats", _i32, [_vp, _vp]),
    ("hdx_alloc_pinned", _i32, [_sz, _vp]),
    ("hdx_free_pinned", _i32, [_vp]),
    ("hdx_synth_lengths", _i32, [ctypes.POINTER(SynthRule), _u32, _u64, _u64, _u64, _vp, _vp]),
    ("hdxdbg_kernel_for", _i32, [_vp, _u32, _u64, ctypes.POINTER(ctypes.c_char_p)]),
    ("hdxdbg_stream_probe", _i32, [_vp, _u64, _vp, _i32, _vp]),
    ("hdxdbg_region_chunk_objects", _u64, [_u64, _u32]),
    ("hdx_synth_fill", _i32, [ctypes.POINTER(SynthRule), _u32, _u64, _u64, _u64, _vp, _vp, _vp,
                              _u64, _vp]),
]

# debug library only (include/hdxhash_debug.h, HDX_DEBUG_BUILD)
DEBUG_SIGNATURES = [
    ("hdxdbg_set_kernel_variant", _i32, [_i32]),
    ("hdxdbg_kernel_variant", _i32, []),
    ("hdxdbg_init_devices", _i32, [_vp, _i32]),
]

_LIB = None
_DEBUG_LIB = None


class HdxError(RuntimeError):
    """A non-OK hdx_status, with the library's hdx_last_error() message."""

    def __init__(self, status, message):
        super().__init__("%s: %s" % (STATUS_NAMES.get(status, status), message))
        self.status = status


def _load(path, signatures):
    if not os.path.exists(path):
        raise ImportError("hyperdex_amd: %s missing — run __graft_entry__.build() "
                          "(make -C hyperdex_amd/csrc)" % path)
    L = ctypes.CDLL(path)
    for name, res, args in signatures:
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def lib():
    """Load libhdxhash.so (raises if it was not built: no silent fallback)."""
    global _LIB
    if _LIB is None:
        _LIB = _load(LIB_PATH, SIGNATURES)
    return _LIB


def debug_lib():
    """libhdxhash_dbg.so: the product's C-ABI plus the A/B kernel selection."""
    global _DEBUG_LIB
    if _DEBUG_LIB is None:
        _DEBUG_LIB = _load(DEBUG_LIB_PATH, SIGNATURES + DEBUG_SIGNATURES)
    return _DEBUG_LIB


@contextlib.contextmanager
def debug_library(variant=None):
    """Route this package's calls through libhdxhash_dbg.so (tests, scripts/),
    optionally with kernel `variant` selected; restores the product library
    and the previous selection on exit."""
    global _LIB
    dbg = debug_lib()
    prev_lib, _LIB = _LIB, dbg
    prev = None
    try:
        if variant is not None:
            prev = dbg.hdxdbg_set_kernel_variant(variant)
            if prev == -2:
                raise ValueError("unknown kernel variant %r" % variant)
        yield dbg
    finally:
        if prev is not None:
            dbg.hdxdbg_set_kernel_variant(prev)
        _LIB = prev_lib


def check(status):
    if status != HDX_OK:
        msg = lib().hdx_last_error()
        raise HdxError(status, msg.decode() if msg else "")
    return status
