"""The reindex sweep from host memory (SURVEY §8 f2, row f2+ of VERDICT r4).

datalayer::indexer_thread::do_work walks a region's stored objects with a
region_iterator (daemon/datalayer_indexer_thread.cc:161-176);
get_from_iterator -> decode_value runs on host bytes read from LevelDB
(daemon/datalayer.cc:853-882).  hdx_hash_encoded_host / _regions_host take
those host arrays, cut them byte-balanced over the device set (the calling
thread's device without one), pipeline each range through PCIe in 128 MiB
chunks and return coordinates, versions and region ids in host memory,
HDX_E_BADENC naming the range of an undecodable value.  Checked against the
oracle's decode_value + hash (oracle/hdx_oracle.c) on the three store
layouts, on a multi-chunk store with a corrupt value in a late chunk, and on
device sets of 2, 3 and 8 workers (repeated ordinals, debug library)."""
import ctypes

import numpy as np
import pytest

import hyperdex_amd as hdx
from hyperdex_amd import _lib, synth


def _store(cfg, n, seed, layout):
    """Host stored objects in one of the three layouts."""
    types, blob, base, lens = synth.make_batch_host(cfg, n, seed=seed)
    if layout == "columns":  # keys in place inside the packed objects
        enc = synth.encode_values_host(types, blob, base, lens, first_version=seed)
    else:
        enc = synth.encode_store_host(types, blob, base, lens, first_version=seed, layout=layout)
    return types, enc


def _pinned_copy(arr):
    """A numpy view of a pinned host copy of arr (freed by the returned closer)."""
    lib = hdx.lib()
    p = ctypes.c_void_p()
    _lib.check(lib.hdx_alloc_pinned(max(arr.nbytes, 1), ctypes.byref(p)))
    buf = (ctypes.c_uint8 * max(arr.nbytes, 1)).from_address(p.value)
    view = np.frombuffer(buf, dtype=arr.dtype, count=arr.size)
    view[:] = arr
    return view, lambda: lib.hdx_free_pinned(p)


def test_host_sweep_arguments_without_device():
    """Validation before any device work: bad schema, NULL arrays."""
    lib = hdx.lib()
    t = np.array([9217, 9218], np.uint32)
    z = np.zeros(4, np.uint64)
    assert lib.hdx_hash_encoded_host(t.ctypes.data, 0, None, 0, z.ctypes.data, z.ctypes.data, None, 0,
                                     z.ctypes.data, z.ctypes.data, 1, z.ctypes.data, None) == _lib.HDX_E_INVALID
    bad = np.array([9217, 12345], np.uint32)
    assert lib.hdx_hash_encoded_host(bad.ctypes.data, 2, None, 0, z.ctypes.data, z.ctypes.data, None, 0,
                                     z.ctypes.data, z.ctypes.data, 1, z.ctypes.data, None) == _lib.HDX_E_BADTYPE
    assert lib.hdx_hash_encoded_host(t.ctypes.data, 2, None, 0, None, z.ctypes.data, None, 0,
                                     z.ctypes.data, z.ctypes.data, 1, z.ctypes.data, None) == _lib.HDX_E_INVALID
    assert lib.hdx_hash_encoded_regions_host(t.ctypes.data, 2, None, 0, z.ctypes.data, z.ctypes.data, None, 0,
                                             z.ctypes.data, z.ctypes.data, 1, None, 0, None, None,
                                             None) == _lib.HDX_E_INVALID
    # n == 0 is a no-op everywhere
    assert lib.hdx_hash_encoded_host(t.ctypes.data, 2, None, 0, None, None, None, 0, None, None, 0, None,
                                     None) == _lib.HDX_OK


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["columns", "keycol", "records"])
@pytest.mark.parametrize("cfg,n", [("cfg3b", 3001), ("mixed", 1500), ("cfg1", 2000), ("wide", 300)])
def test_gpu_host_sweep_layouts(oracle, cfg, n, layout):
    types, enc = _store(cfg, n, n + 11, layout)
    want, wver, bad = oracle.hash_encoded(types, *enc)
    assert not bad.any()
    c, v = hdx.hash_encoded_host(types, *enc, versions=True)
    assert np.array_equal(c, want)
    assert np.array_equal(v, wver)


@pytest.mark.gpu
def test_gpu_host_sweep_pinned_inputs(oracle):
    """Pinned keys / values / lengths (no staging copies) give the same result."""
    types, enc = _store("cfg3b", 5000, 3, "keycol")
    want, wver, _ = oracle.hash_encoded(types, *enc)
    pinned, closers = [], []
    for a in enc:
        view, close = _pinned_copy(np.ascontiguousarray(a))
        pinned.append(view)
        closers.append(close)
    try:
        c, v = hdx.hash_encoded_host(types, *pinned, versions=True)
    finally:
        for close in closers:
            close()
    assert np.array_equal(c, want) and np.array_equal(v, wver)


def _big_store(layout, n, seed):
    """~1.25 KB config-3b objects encoded in HBM (synth.make_encoded_device) and
    copied to host memory."""
    import torch
    dev = torch.device("cuda", 0)
    types, keys, ko, kl, vals, vo, vl = synth.make_encoded_device("cfg3b", n, seed=seed, device=dev, layout=layout)
    torch.cuda.synchronize()
    hk = keys.cpu().numpy()
    hv = hk if layout == "records" else vals.cpu().numpy()
    enc = (hk, ko.cpu().numpy().view(np.uint64), kl.cpu().numpy().view(np.uint32), hv,
           vo.cpu().numpy().view(np.uint64), vl.cpu().numpy().view(np.uint32))
    del keys, vals, ko, kl, vo, vl
    torch.cuda.empty_cache()
    return types, enc


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["keycol", "records"])
def test_gpu_host_sweep_multichunk_late_corrupt(oracle, layout):
    """A store of ≈ 440 MB (four 128 MiB pipeline chunks) with one value
    corrupted in the last chunk: HDX_E_BADENC with the range named, that
    object's coordinates and version zero, every other object exact."""
    n = 400_000
    types, enc = _big_store(layout, n, seed=23)
    keys, ko, kl, vals, vo, vl = enc
    assert vals.nbytes > 3 * (128 << 20)
    vals = vals.copy() if layout != "records" else vals
    victim = n - 1234
    vals[int(vo[victim]) + 9] ^= 3  # the count no longer equals A - 1
    keys = vals if layout == "records" else keys
    enc = (keys, ko, kl, vals, vo, vl)
    want, wver, bad = oracle.hash_encoded(types, *enc)
    assert list(np.nonzero(bad)[0]) == [victim]
    c, v, st, msg = hdx.hash_encoded_host_status(types, *enc)
    assert st == _lib.HDX_E_BADENC and "decode" in msg, msg
    assert np.array_equal(c, want)
    assert np.array_equal(v, wver)
    assert (c[victim] == 0).all() and v[victim] == 0


@pytest.mark.gpu
def test_gpu_host_sweep_regions(oracle):
    """hdx_hash_encoded_regions_host: each object's region in two subspaces,
    with and without the coordinates."""
    from hyperdex_amd import RegionTable
    types, enc = _store("cfg3b", 4000, 9, "records")
    want, wver, _ = oracle.hash_encoded(types, *enc)
    specs = [([0],) + tuple(oracle.partition(1, 64)), ([1, 2, 3],) + tuple(oracle.partition(3, 64))]
    tables = [RegionTable(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 3) for at, lo, up in specs]
    c, v, st, msg, ids = hdx.hash_encoded_host_status(types, *enc, tables=tables)
    assert st == _lib.HDX_OK, msg
    assert np.array_equal(c, want) and np.array_equal(v, wver)
    for k, (at, lo, up) in enumerate(specs):
        assert np.array_equal(ids[k], oracle.lookup_region(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 3,
                                                          want))
    # without coordinates (NULL coords through the C-ABI)
    lib = hdx.lib()
    t = np.asarray(types, np.uint32)
    keys, ko, kl, vals, vo, vl = [np.ascontiguousarray(a) for a in enc]
    ids2 = np.zeros((2, len(vo)), np.uint64)
    handles = (ctypes.c_void_p * 2)(*[tb.handle.value for tb in tables])
    _lib.check(lib.hdx_hash_encoded_regions_host(t.ctypes.data, len(t), keys.ctypes.data, keys.size, ko.ctypes.data,
                                                 kl.ctypes.data, keys.ctypes.data, keys.size, vo.ctypes.data,
                                                 vl.ctypes.data, len(vo), handles, 2, ids2.ctypes.data, None, None))
    assert np.array_equal(ids2, ids)
    for tb in tables:
        tb.close()


@pytest.mark.gpu
def test_gpu_host_sweep_through_the_set(oracle):
    """After hdx_init_mask the sweep is cut over the set; the calling thread
    runs its own device's range (set {0} on the one-GPU box)."""
    types, enc = _store("cfg3b", 6000, 4, "keycol")
    want, wver, _ = oracle.hash_encoded(types, *enc)
    hdx.init_mask(1)
    try:
        c, v = hdx.hash_encoded_host(types, *enc, versions=True)
    finally:
        hdx.shutdown()
    assert np.array_equal(c, want) and np.array_equal(v, wver)


@pytest.fixture(params=[2, 3, 8])
def repeated_set(request):
    import torch
    assert torch.cuda.is_available()
    world = request.param
    with _lib.debug_library() as dbg:
        devs = (ctypes.c_int * world)(*([0] * world))
        assert dbg.hdxdbg_init_devices(devs, world) == _lib.HDX_OK
        yield world
        hdx.shutdown()


@pytest.mark.gpu
def test_gpu_host_sweep_repeated_set(oracle, repeated_set):
    """`world` byte-balanced ranges (key + value bytes), one per worker (the
    caller runs the first), each its own pipeline: bit-exact; a corrupt value
    in the last range fails that range with the device named while every
    other object is hashed."""
    world = repeated_set
    types, enc = _store("cfg3b", 20_003, 61, "records")
    want, wver, _ = oracle.hash_encoded(types, *enc)
    c, v = hdx.hash_encoded_host(types, *enc, versions=True)
    assert np.array_equal(c, want) and np.array_equal(v, wver)
    keys, ko, kl, vals, vo, vl = enc
    vals = vals.copy()
    victim = 20_000
    vals[int(vo[victim]) + 9] ^= 1
    enc2 = (vals, ko, kl, vals, vo, vl)
    want2, wver2, bad = oracle.hash_encoded(types, *enc2)
    c2, v2, st, msg = hdx.hash_encoded_host_status(types, *enc2)
    assert st == _lib.HDX_E_BADENC and "device 0" in msg, msg
    assert np.array_equal(c2, want2) and np.array_equal(v2, wver2)
