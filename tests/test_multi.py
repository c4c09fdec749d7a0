"""The device set of hdx_init_mask (hyperdex_amd/csrc/hdx_multi.cpp): the C++
byte-balanced cut rule against hyperdex_amd.dist.shard_ranges, the
host-resident batch split over the set's devices, and
hdx_hash_batch_device_multi with its in-process RCCL gather — everything a
C++ daemon (daemon/daemon.cc:345-351 -> key_state::hash_objects,
daemon/key_state.cc:1455-1543) reaches without Python or torch.

On the one-GPU test box the set is {0}: the workers, the cuts, the shard
arguments and RCCL (a communicator of one) all run; 2..8 devices are the
driver's 8-GPU node."""
import ctypes
import os
import subprocess
import threading

import numpy as np
import pytest

import hyperdex_amd as hdx
from hyperdex_amd import _lib, dist, hashing, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---- CPU: the cut rule ---------------------------------------------------------

def _sizes(lens, n, A):
    return lens.reshape(n, A).astype(np.uint64).sum(axis=1) if n else np.zeros(0)


@pytest.mark.parametrize("n,A,world,tol", [
    (0, 3, 4, 0.0), (1, 3, 4, 0.0), (3, 2, 8, 0.0), (10, 1, 3, 0.0), (65535, 2, 2, 0.0), (65536, 2, 3, 0.0),
    (65537, 2, 5, 0.0), (300_000, 3, 5, 0.0), (300_000, 3, 7, 1e-3), (300_000, 3, 7, 1e-9),
    (200_000, 17, 8, 0.0), (200_000, 17, 8, 1e-3), (131_073, 5, 1, 0.0)])
def test_cut_rule_matches_dist(n, A, world, tol):
    """hdx_shard_ranges gives exactly dist.shard_ranges' cuts: ragged n, every
    block boundary of the C++ prefix (2^16 objects), runs of empty objects,
    and both sides of the equal-count tolerance."""
    rng = np.random.default_rng(n * 31 + world)
    lens = rng.integers(0, 200, size=n * A).astype(np.uint32)
    if n > 5:
        lens[:(n // 3) * A] = 0  # a third of the objects empty: cuts must skip them alike
        lens[(n // 2) * A:(n // 2 + 7) * A] = 100_000  # a few huge objects
    got = hashing.shard_ranges(lens, A, n, world, tol)
    want = dist.shard_ranges(n, world, _sizes(lens, n, A), tol)
    assert got == want
    assert sum(c for _, c in got) == n


def test_cut_rule_skewed_and_equal_counts():
    """One object holding most of the bytes; no sizes = counts differing by <= 1."""
    n, A = 1000, 2
    lens = np.ones(n * A, np.uint32)
    lens[500 * A] = 10 ** 9
    for world in (2, 3, 8):
        assert hashing.shard_ranges(lens, A, n, world) == dist.shard_ranges(n, world, _sizes(lens, n, A))
        assert hashing.shard_ranges(None, A, n, world) == dist.shard_ranges(n, world)


def test_multi_arguments_without_a_set():
    lib = hdx.lib()
    first = np.zeros(3, np.uint64)
    assert lib.hdx_shard_ranges(None, 1, 10, 0, 0.0, first.ctypes.data) == _lib.HDX_E_INVALID
    assert lib.hdx_shard_ranges(None, 1, 10, 2, 0.0, None) == _lib.HDX_E_INVALID
    t = np.array([9217], np.uint32)
    if not hdx.device_set():
        shards = (_lib.Shard * 1)()
        assert lib.hdx_hash_batch_device_multi(t.ctypes.data, 1, shards, 1, 1) == _lib.HDX_E_INVALID
        assert b"hdx_init_mask" in lib.hdx_last_error()
    assert lib.hdx_hash_batch_device_multi(None, 1, None, 0, 1) == _lib.HDX_E_INVALID


# ---- GPU: the set {0} ------------------------------------------------------------

@pytest.fixture()
def device_set0():
    import torch
    assert torch.cuda.is_available()
    hdx.init_mask(1)
    assert hdx.device_set() == [0]
    yield torch
    hdx.shutdown()
    assert hdx.device_set() == []


@pytest.mark.gpu
def test_host_batch_through_the_set(oracle, device_set0):
    """hdx_hash_batch_host after hdx_init_mask: cut, posted to the device's
    worker, pipelined into the caller's rows — bit-exact, from several
    caller threads at once, and across a shutdown / re-init."""
    types, blob, base, lens = synth.make_batch_host("cfg3b", 20_000, seed=41)
    want, _ = oracle.hash_batch(types, blob, base, lens)
    assert np.array_equal(hdx.hash_batch_host(types, blob, base, lens), want)
    outs, errs = [None] * 4, []

    def run(k):
        try:
            outs[k] = hdx.hash_batch_host(types, blob, base, lens)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ths = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errs and all(np.array_equal(o, want) for o in outs)
    hdx.shutdown()
    assert hdx.hash_batch_host(types, blob, base, lens).tobytes() == want.tobytes()  # no set: caller's device
    hdx.init_mask(1)
    assert np.array_equal(hdx.hash_batch_host(types, blob, base, lens), want)


@pytest.mark.gpu
def test_host_batch_set_multichunk_and_bad_size(oracle, device_set0):
    """A 326 MB batch (three 128 MiB pipeline chunks) through the set, sampled
    against the oracle; a mis-sized numeric fails with HDX_E_BADSIZE and the
    device named in the message."""
    types, blob, base, lens = synth.make_batch_host("cfg3a", 300_000, seed=8)
    got = hdx.hash_batch_host(types, blob, base, lens)
    idx = np.sort(np.random.default_rng(0).choice(len(base), 3000, replace=False))
    want, _ = oracle.hash_batch(types, blob, base[idx], lens.reshape(len(base), -1)[idx].ravel())
    assert np.array_equal(got[idx], want)
    types, blob, base, lens = synth.make_batch_host("cfg2", 50_000, seed=9)
    lens = lens.copy()
    lens[40_000 * len(types) + 2] = 5
    with pytest.raises(hdx.HdxError) as e:
        hdx.hash_batch_host(types, blob, base, lens)
    assert e.value.status == _lib.HDX_E_BADSIZE and "device 0" in str(e.value)


def _dev_batch(torch, cfg, n, seed):
    dev = torch.device("cuda", 0)
    return synth.make_batch_device(cfg, n, seed=seed, device=dev)


@pytest.mark.gpu
@pytest.mark.parametrize("gather", [True, False])
@pytest.mark.parametrize("cfg,n", [("cfg3b", 50_001), ("cfg2", 70_000), ("cfg3a", 1), ("mixed", 0)])
def test_device_multi_matches_oracle(oracle, device_set0, cfg, n, gather):
    """hdx_hash_batch_device_multi over the set {0}: the shard hashed into its
    rows, then (gather) the in-place all-gather over RCCL — a communicator of
    one device — bit-exact against the oracle; empty shards are no-ops."""
    torch = device_set0
    types, blob, base, lens = _dev_batch(torch, cfg, n, seed=n + 5)
    status = torch.zeros(1, dtype=torch.int32, device=base.device)
    (c,) = hdx.hash_batch_device_multi(types, [(blob, base, lens, status)], gather=gather)
    assert c.shape == (n, len(types))
    if n:
        want, _ = oracle.hash_batch(types, blob.cpu().numpy(), base.cpu().numpy().view(np.uint64),
                                    lens.cpu().numpy().view(np.uint32))
        assert np.array_equal(c.cpu().numpy().view(np.uint64), want)
    assert int(status.item()) == 0


@pytest.mark.gpu
def test_device_multi_rejects_wrong_shards(device_set0):
    """Shard count != set size, a NULL pointer, and a bad numeric size through
    the status word."""
    torch = device_set0
    types, blob, base, lens = _dev_batch(torch, "cfg2", 1000, seed=3)
    lib = hdx.lib()
    t = np.asarray(types, np.uint32)
    two = (_lib.Shard * 2)()
    assert lib.hdx_hash_batch_device_multi(t.ctypes.data, len(t), two, 2, 1) == _lib.HDX_E_INVALID
    one = (_lib.Shard * 1)(_lib.Shard(blob.data_ptr(), None, lens.data_ptr(), 1000, None, None))
    assert lib.hdx_hash_batch_device_multi(t.ctypes.data, len(t), one, 1, 1) == _lib.HDX_E_INVALID
    lens2 = lens.clone()
    lens2[17 * len(types) + 1] = 3
    status = torch.zeros(1, dtype=torch.int32, device=base.device)
    hdx.hash_batch_device_multi(types, [(blob, base, lens2, status)], gather=True)
    assert int(status.item()) == 1 << _lib.HDX_E_BADSIZE


MULTI_EXE = os.path.join(ROOT, "tests", "cpp", "multi_test")


@pytest.mark.gpu
def test_cpp_daemon_uses_every_device():
    """tests/cpp/multi_test.cc, a C++ caller with no Python or torch: binds
    every visible gfx950 device with hdx_init_mask, hashes a host batch from 4
    threads at once and a device-resident batch sharded over the set with the
    RCCL gather, and checks both against the product's per-object CPU path
    (hdx_hash_object).  Built by __graft_entry__.build()."""
    assert os.path.exists(MULTI_EXE), "tests/cpp/multi_test missing: run __graft_entry__.build()"
    r = subprocess.run([MULTI_EXE, "200000"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "multi ok" in r.stdout, r.stdout


# ---- world 2, 3 and 8 on one GPU (debug library: a device set listing device 0 repeatedly) ----

@pytest.fixture(params=[2, 3, 8])
def repeated_set(request):
    """hdxdbg_init_devices([0] * world): `world` workers and streams on device 0,
    so the multi-device cuts, the per-device workers and the shard plumbing
    run at world > 1 on the one-GPU box."""
    import torch
    assert torch.cuda.is_available()
    world = request.param
    with _lib.debug_library() as dbg:
        devs = (ctypes.c_int * world)(*([0] * world))
        assert dbg.hdxdbg_init_devices(devs, world) == _lib.HDX_OK
        assert hdx.device_set() == [0] * world
        yield torch, world
        hdx.shutdown()


@pytest.mark.gpu
def test_host_batch_split_over_repeated_set(oracle, repeated_set):
    """hdx_hash_batch_host cut into `world` byte-balanced ranges, one per
    worker: bit-exact, also for a multi-chunk batch and a bad size in the last
    range (its error, after the other ranges ran)."""
    torch, world = repeated_set
    types, blob, base, lens = synth.make_batch_host("cfg3b", 30_001, seed=61)
    want, _ = oracle.hash_batch(types, blob, base, lens)
    assert np.array_equal(hdx.hash_batch_host(types, blob, base, lens), want)
    types, blob, base, lens = synth.make_batch_host("cfg3a", 300_000, seed=62)  # ~326 MB: chunks per range
    got = hdx.hash_batch_host(types, blob, base, lens)
    idx = np.sort(np.random.default_rng(3).choice(len(base), 3000, replace=False))
    w2, _ = oracle.hash_batch(types, blob, base[idx], lens.reshape(len(base), -1)[idx].ravel())
    assert np.array_equal(got[idx], w2)
    types, blob, base, lens = synth.make_batch_host("cfg2", 60_000, seed=63)
    lens = lens.copy()
    lens[59_990 * len(types) + 1] = 3
    out = np.zeros((len(base), len(types)), np.uint64)
    with pytest.raises(hdx.HdxError) as e:
        hdx.hash_batch_host(types, blob, base, lens, out=out)
    assert e.value.status == _lib.HDX_E_BADSIZE
    first = hashing.shard_ranges(lens, len(types), len(base), world)[0]
    w3, _ = oracle.hash_batch(types, blob, base[:first[1]], lens[:first[1] * len(types)])
    assert np.array_equal(out[:first[1]], w3.reshape(first[1], -1))  # range 0 ran to completion


@pytest.mark.gpu
def test_device_shards_over_repeated_set(oracle, repeated_set):
    """hdx_hash_batch_device_multi with `world` shards cut by hdx_shard_ranges
    (unequal counts), ungathered: every shard's rows bit-exact; a gather over
    a repeated device is refused before RCCL is touched."""
    torch, world = repeated_set
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_host("cfg3b", 40_003, seed=64)
    A = len(types)
    want, _ = oracle.hash_batch(types, blob, base, lens)
    ranges = hashing.shard_ranges(lens, A, len(base), world)
    assert len(set(c for _, c in ranges)) > 1  # byte-balanced: unequal counts
    shards = []
    for f, c in ranges:
        sb = base[f:f + c]
        lo = int(sb[0])
        hi = int(sb[-1] + lens[(f + c - 1) * A:(f + c) * A].astype(np.uint64).sum())
        shards.append((torch.from_numpy(blob[lo:hi].copy()).to(dev),
                       torch.from_numpy((sb - np.uint64(lo)).view(np.int64).copy()).to(dev),
                       torch.from_numpy(lens[f * A:(f + c) * A].view(np.int32).copy()).to(dev)))
    outs = hdx.hash_batch_device_multi(types, shards, gather=False)
    for (f, c), o in zip(ranges, outs):
        assert np.array_equal(o.cpu().numpy().view(np.uint64), want[f:f + c])
    with pytest.raises(hdx.HdxError) as e:
        hdx.hash_batch_device_multi(types, shards, gather=True)
    assert e.value.status == _lib.HDX_E_INVALID


# ---- region ids: host batches and device shards (VERDICT r4 "do this" #1) ------------

def _tables(oracle, A):
    from hyperdex_amd import RegionTable
    specs = [([0],) + tuple(oracle.partition(1, 64)), ([1, 2, A - 1],) + tuple(oracle.partition(3, 27))]
    return specs, [RegionTable(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 11) for at, lo, up in specs]


def _want_ids(oracle, specs, coords):
    return np.stack([oracle.lookup_region(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 11, coords)
                     for at, lo, up in specs])


@pytest.mark.gpu
@pytest.mark.parametrize("use_set", [False, True])
def test_host_regions_batch(oracle, use_set):
    """hdx_hash_batch_regions_host: host batch in, region ids (and optionally
    coordinates) out, without a set and through the set {0}; 8 bytes per
    table per object come back over PCIe instead of 8 * A."""
    import torch
    assert torch.cuda.is_available()
    types, blob, base, lens = synth.make_batch_host("cfg3b", 30_001, seed=71)
    want, _ = oracle.hash_batch(types, blob, base, lens)
    specs, tables = _tables(oracle, len(types))
    wids = _want_ids(oracle, specs, want)
    if use_set:
        hdx.init_mask(1)
    try:
        ids = hdx.hash_batch_regions_host(types, blob, base, lens, tables)
        ids2, c = hdx.hash_batch_regions_host(types, blob, base, lens, tables, coords=True)
    finally:
        if use_set:
            hdx.shutdown()
    assert np.array_equal(ids, wids) and np.array_equal(ids2, wids) and np.array_equal(c, want)
    for t in tables:
        t.close()


@pytest.mark.gpu
@pytest.mark.parametrize("gather", [True, False])
@pytest.mark.parametrize("cfg,n", [("cfg3b", 40_001), ("cfg2", 9_000), ("cfg3a", 1)])
def test_device_multi_regions_set0(oracle, device_set0, cfg, n, gather):
    """hdx_hash_batch_regions_device_multi over the set {0}: region ids
    (gathered: the plan's in-place all-gather per table over a communicator
    of one) equal to the oracle's lookup_region of the oracle's coordinates;
    the shard's own coordinates when asked."""
    torch = device_set0
    types, blob, base, lens = _dev_batch(torch, cfg, n, seed=n + 9)
    want, _ = oracle.hash_batch(types, blob.cpu().numpy(), base.cpu().numpy().view(np.uint64),
                                lens.cpu().numpy().view(np.uint32))
    specs, tables = _tables(oracle, len(types))
    wids = _want_ids(oracle, specs, want)
    (ids,), (c,) = hdx.hash_batch_regions_device_multi(types, [(blob, base, lens)], tables, gather=gather,
                                                       coords=True)
    assert np.array_equal(ids.cpu().numpy().view(np.uint64), wids)
    assert np.array_equal(c.cpu().numpy().view(np.uint64), want)
    (ids2,) = hdx.hash_batch_regions_device_multi(types, [(blob, base, lens)], tables, gather=gather)
    assert np.array_equal(ids2.cpu().numpy().view(np.uint64), wids)
    for t in tables:
        t.close()


@pytest.mark.gpu
def test_host_regions_and_shards_over_repeated_set(oracle, repeated_set):
    """World 2, 3 and 8 (repeated ordinals): the host regions batch cut over
    the set (the caller runs range 0), and ungathered region-id shards of
    unequal counts; a gather over a repeated device is refused before any
    launch."""
    torch, world = repeated_set
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_host("cfg3b", 30_007, seed=83)
    A = len(types)
    want, _ = oracle.hash_batch(types, blob, base, lens)
    specs, tables = _tables(oracle, A)
    wids = _want_ids(oracle, specs, want)
    assert np.array_equal(hdx.hash_batch_regions_host(types, blob, base, lens, tables), wids)
    ranges = hashing.shard_ranges(lens, A, len(base), world)
    shards = []
    for f, c in ranges:
        sb = base[f:f + c]
        lo = int(sb[0])
        hi = int(sb[-1] + lens[(f + c - 1) * A:(f + c) * A].astype(np.uint64).sum())
        shards.append((torch.from_numpy(blob[lo:hi].copy()).to(dev),
                       torch.from_numpy((sb - np.uint64(lo)).view(np.int64).copy()).to(dev),
                       torch.from_numpy(lens[f * A:(f + c) * A].view(np.int32).copy()).to(dev)))
    outs = hdx.hash_batch_regions_device_multi(types, shards, tables, gather=False)
    for (f, c), o in zip(ranges, outs):
        assert np.array_equal(o.cpu().numpy().view(np.uint64), wids[:, f:f + c])
    with pytest.raises(hdx.HdxError) as e:
        hdx.hash_batch_regions_device_multi(types, shards, tables, gather=True)
    assert e.value.status == _lib.HDX_E_INVALID and "twice" in str(e.value)
    for t in tables:
        t.close()


THREAD_EXE = os.path.join(ROOT, "tests", "cpp", "thread_exit_test")


@pytest.mark.gpu
def test_threads_exit_without_shutdown(tmp_path):
    """tests/cpp/thread_exit_test.cc: daemon-style threads use the host batch,
    the host sweep and the search, then exit without hdx_shutdown — three
    rounds of fresh threads, the process ends without hdx_shutdown.  Plain and
    under rocprofv3 --kernel-trace (round 4's abort: HIP calls in
    thread-local destructors after the profiler's per-thread state was gone;
    now the destructors park the frees and make no HIP call)."""
    import shutil
    assert os.path.exists(THREAD_EXE), "tests/cpp/thread_exit_test missing: run __graft_entry__.build()"
    r = subprocess.run([THREAD_EXE, "20000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "thread_exit ok" in r.stdout, r.stdout + r.stderr
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        pytest.skip("rocprofv3 not installed")
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run([prof, "--kernel-trace", "-d", str(tmp_path / "prof"), "-o", "trace", "--", THREAD_EXE,
                        "5000"], capture_output=True, text=True, timeout=240, cwd=str(tmp_path), env=env)
    assert r.returncode == 0 and "thread_exit ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("form", ["coords", "regions"])
def test_gather_between_distinct_devices(oracle, form):
    """the RCCL exchange between distinct devices — unequal
    byte-balanced shards (the grouped in-place broadcasts) and equal counts
    (the in-place all-gather), every device's whole matrix against the
    oracle.  Needs two or more GPUs: skipped on the one-GPU test boxes (the
    driver's 8-GPU node runs it)."""
    import torch
    ndev = hdx.lib().hdx_device_count()
    if ndev < 2:
        pytest.skip("one GPU: the exchange between distinct devices needs two or more")
    world = min(ndev, 8)
    hdx.init_mask((1 << world) - 1)
    try:
        types, blob, base, lens = synth.make_batch_host("cfg3b", 50_003, seed=97)
        A = len(types)
        want, _ = oracle.hash_batch(types, blob, base, lens)
        specs, tables = _tables(oracle, A)
        wids = _want_ids(oracle, specs, want)
        for tol in (0.0, 1e-3):  # byte-balanced (unequal counts), then equal counts
            ranges = hashing.shard_ranges(lens, A, len(base), world, tol)
            shards = []
            for k, (f, c) in enumerate(ranges):
                d = torch.device("cuda", k)
                sb = base[f:f + c]
                lo = int(sb[0]) if c else 0
                hi = int(sb[-1] + lens[(f + c - 1) * A:(f + c) * A].astype(np.uint64).sum()) if c else 0
                shards.append((torch.from_numpy(blob[lo:hi + 1].copy()).to(d),
                               torch.from_numpy((sb - np.uint64(lo)).view(np.int64).copy()).to(d),
                               torch.from_numpy(lens[f * A:(f + c) * A].view(np.int32).copy()).to(d)))
            if form == "coords":
                outs = hdx.hash_batch_device_multi(types, shards, gather=True)
                for o in outs:
                    assert np.array_equal(o.cpu().numpy().view(np.uint64), want)
            else:
                outs = hdx.hash_batch_regions_device_multi(types, shards, tables, gather=True)
                for o in outs:
                    assert np.array_equal(o.cpu().numpy().view(np.uint64), wids)
        for t in tables:
            t.close()
    finally:
        hdx.shutdown()
