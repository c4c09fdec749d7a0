"""Region lookup (configuration::lookup_region): oracle semantics
on CPU, GPU kernel vs oracle on partition() grids and adversarial tables."""
import contextlib

import numpy as np
import pytest

from hyperdex_amd import synth

U64MAX = np.uint64(0xffffffffffffffff)


def test_partition_matches_reference_counts(oracle):
    """admin/partition.cc quirk (partitions = dims.size()*dims[0], :109)."""
    counts = {(1, 64): 64, (16, 64): 4, (3, 8): 12, (3, 64): 64}
    for (a, s), want in counts.items():
        lo, up = oracle.partition(a, s)
        assert len(lo) == want
        # every cell tiles: per dimension the intervals start at 0 and end at 2^64-1
        assert lo[:, 0].min() == 0 and up[:, 0].max() == U64MAX


def test_lookup_semantics_first_match_inclusive(oracle):
    attrs = [2]
    lower = np.array([[10], [0], [5]], np.uint64)
    upper = np.array([[20], [100], [15]], np.uint64)
    ids = np.array([7, 8, 9], np.uint64)
    coords = np.zeros((6, 3), np.uint64)
    coords[:, 2] = [10, 20, 5, 21, 100, 101]
    got = oracle.lookup_region(attrs, lower, upper, ids, coords)
    assert list(got) == [7, 7, 8, 8, 8, 0]  # first match wins; inclusive; none -> 0


def _grid_table(oracle, dims, servers, attrs, first_id=10):
    lo, up = oracle.partition(dims, servers)
    ids = np.arange(first_id, first_id + len(lo), dtype=np.uint64)
    return attrs, lo, up, ids


def _coords(rng, n, A, lo, up, attrs):
    c = rng.integers(0, 2**64, size=(n, A), dtype=np.uint64)
    # a quarter of the rows sit exactly on region boundaries
    k = n // 4
    for d, a in enumerate(attrs):
        pick = rng.integers(0, len(lo), k)
        c[:k // 2, a] = lo[pick[:k // 2], d]
        c[k // 2:k, a] = up[pick[k // 2:], d]
    c[0, :] = 0
    c[1, :] = U64MAX
    return c


@pytest.mark.gpu
@pytest.mark.parametrize("dims,servers,A", [(1, 64, 17), (3, 64, 17), (2, 256, 5), (16, 64, 17),
                                            (1, 1, 1), (4, 100, 9)])
def test_gpu_lookup_matches_oracle_on_grids(oracle, dims, servers, A):
    import torch

    from hyperdex_amd import regions
    rng = np.random.default_rng(dims * 1000 + servers)
    attrs = list(rng.choice(A, size=dims, replace=False)) if dims <= A else None
    attrs, lo, up, ids = _grid_table(oracle, dims, servers, attrs)
    coords = _coords(rng, 20000, A, lo, up, attrs)
    want = oracle.lookup_region(attrs, lo, up, ids, coords)
    t = regions.RegionTable(attrs, lo, up, ids)
    dev = torch.device("cuda", 0)
    got = regions.lookup_region(t, torch.from_numpy(coords.view(np.int64)).to(dev))
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [1, 7, 300, 2500])
def test_gpu_lookup_overlapping_boxes(oracle, R):
    """Random overlapping boxes with gaps: first-match order and region_id() = 0
    must follow the table order exactly (R=2500, D=3 exceeds the LDS path)."""
    import torch

    from hyperdex_amd import regions
    rng = np.random.default_rng(R)
    A, attrs = 6, [5, 0, 3]
    a = rng.integers(0, 2**64, size=(R, 3), dtype=np.uint64)
    b = rng.integers(0, 2**64, size=(R, 3), dtype=np.uint64)
    lo, up = np.minimum(a, b), np.maximum(a, b)
    ids = rng.integers(1, 2**63, R, dtype=np.uint64)
    coords = _coords(rng, 30000, A, lo, up, attrs)
    want = oracle.lookup_region(attrs, lo, up, ids, coords)
    assert (want == 0).any() or R < 50
    t = regions.RegionTable(attrs, lo, up, ids)
    got = regions.lookup_region(t, torch.from_numpy(coords.view(np.int64)).to(torch.device("cuda", 0)))
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [2, 63, 64, 65, 200, 256])
@pytest.mark.parametrize("scan", [False, True])
def test_gpu_lookup_index_vs_scan(oracle, R, scan, monkeypatch):
    """The interval index (tables of <= 256 regions) and the box scan
    (HDX_REGION_SCAN=1) agree with the oracle's first-match scan on
    overlapping boxes, empty boxes (lower > upper), boxes reaching 0 and
    2^64-1, and duplicated boxes (first one wins)."""
    import torch

    import contextlib

    from hyperdex_amd import _lib, regions
    if scan:  # an A/B switch of the debug library only
        monkeypatch.setenv("HDX_REGION_SCAN", "1")
    rng = np.random.default_rng(R + 7)
    A, attrs = 9, [8, 2]
    a = rng.integers(0, 2**64, size=(R, 2), dtype=np.uint64)
    b = rng.integers(0, 2**64, size=(R, 2), dtype=np.uint64)
    lo, up = np.minimum(a, b), np.maximum(a, b)
    lo[0, 0] = 0
    up[R // 2, 1] = U64MAX
    if R > 3:
        lo[1], up[1] = up[1], lo[1]          # empty box on both dimensions
        lo[R - 1], up[R - 1] = lo[2], up[2]  # duplicate of box 2: never the first match
    ids = rng.integers(1, 2**63, R, dtype=np.uint64)
    coords = _coords(rng, 20000, A, lo, up, attrs)
    want = oracle.lookup_region(attrs, lo, up, ids, coords)
    with _lib.debug_library() if scan else contextlib.nullcontext():
        t = regions.RegionTable(attrs, lo, up, ids)
        got = regions.lookup_region(t, torch.from_numpy(coords.view(np.int64)).to(torch.device("cuda", 0)))
        torch.cuda.synchronize()
        t.close()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [40, 256])
def test_gpu_lookup_clustered_boundaries(oracle, R):
    """The index's top-byte buckets (hdx_regions.hip region_index_build): box
    edges crowded into two top-byte values (up to 2R boundaries in one bucket:
    a multi-step search inside it), edges exactly on bucket starts (b << 56)
    and one below, coordinates on and beside every edge."""
    import torch

    from hyperdex_amd import regions
    rng = np.random.default_rng(R)
    A, attrs = 4, [3, 1]
    base = np.array([0x12 << 56, 0xfe << 56], np.uint64)
    a = base[rng.integers(0, 2, size=(R, 2))] + rng.integers(0, 1 << 56, size=(R, 2), dtype=np.uint64)
    b = base[rng.integers(0, 2, size=(R, 2))] + rng.integers(0, 1 << 56, size=(R, 2), dtype=np.uint64)
    lo, up = np.minimum(a, b), np.maximum(a, b)
    lo[0, 0], up[0, 0] = np.uint64(0x40 << 56), np.uint64((0x41 << 56) - 1)
    lo[1, 1], up[1, 1] = np.uint64(0x41 << 56), U64MAX
    ids = rng.integers(1, 2**63, R, dtype=np.uint64)
    edges = np.concatenate([lo.ravel(), up.ravel(), up.ravel() + np.uint64(1), lo.ravel() - np.uint64(1)])
    coords = rng.integers(0, 2**64, size=(40000, A), dtype=np.uint64)
    for a_ in attrs:
        coords[:30000, a_] = edges[rng.integers(0, len(edges), 30000)]
    want = oracle.lookup_region(attrs, lo, up, ids, coords)
    t = regions.RegionTable(attrs, lo, up, ids)
    got = regions.lookup_region(t, torch.from_numpy(coords.view(np.int64)).to(torch.device("cuda", 0)))
    torch.cuda.synchronize()
    t.close()
    assert (want != 0).sum() > 1000
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)


@pytest.mark.gpu
def test_gpu_hash_then_point_leader(oracle):
    """hash -> lookup on subspace 0 (point_leader's region step) end to end."""
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import regions, synth
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_device("cfg3b", 50000, device=dev)
    coords = hdx.hash_batch(types, blob, base, lens)
    lo, up = oracle.partition(1, 64)
    ids = np.arange(2, 66, dtype=np.uint64)
    got = regions.lookup_region(regions.RegionTable([0], lo, up, ids), coords)
    torch.cuda.synchronize()
    want = oracle.lookup_region([0], lo, up, ids, coords.cpu().numpy().view(np.uint64))
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)
    assert (want != 0).all()  # the key grid covers the whole space


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,n,with_coords", [("cfg3a", 3001, False), ("cfg3b", 2999, True), ("cfg2", 4097, False),
                                               ("mixed", 1000, True), ("cfg1", 65, True), ("cfg3b", 1, False)])
def test_gpu_batch_regions_fused(oracle, cfg, n, with_coords):
    """hdx_hash_batch_regions_device = hash_batch's coordinates looked up in
    every table (indexed key grid, indexed 3-attribute grid, a scanned
    300-region table), with and without the coordinates written."""
    import numpy as np
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import RegionTable, synth
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_host(cfg, n, seed=n + 17)
    want_coords, _ = oracle.hash_batch(types, blob, base, lens)
    A = len(types)
    rng = np.random.default_rng(n)
    lo1, up1 = oracle.partition(1, 64)
    specs = [([0], lo1, up1)]
    if A >= 4:
        lo3, up3 = oracle.partition(3, 64)
        specs.append(([1, 2, 3], lo3, up3))
    a = rng.integers(0, 2**64, size=(300, 2), dtype=np.uint64)
    b = rng.integers(0, 2**64, size=(300, 2), dtype=np.uint64)
    specs.append(([A - 1, 0], np.minimum(a, b), np.maximum(a, b)))
    tables = [RegionTable(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 3) for at, lo, up in specs]
    d_blob = torch.from_numpy(np.ascontiguousarray(blob) if len(blob) else np.zeros(1, np.uint8)).to(dev)
    d_base = torch.from_numpy(base.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = hdx.hash_batch_regions(types, d_blob, d_base, d_lens, tables, coords=with_coords)
    torch.cuda.synchronize()
    ids, coords = out if with_coords else (out, None)
    for k, (at, lo, up) in enumerate(specs):
        want = oracle.lookup_region(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 3, want_coords)
        assert np.array_equal(ids[k].cpu().numpy().view(np.uint64), want), k
    if with_coords:
        assert np.array_equal(coords.cpu().numpy().view(np.uint64), want_coords)
    for t in tables:
        t.close()


WIDE_MIXED = ([synth.Rule(synth.dt.HYPERDATATYPE_STRING, synth.UNIFORM, 0, 40),
               synth.Rule(synth.dt.HYPERDATATYPE_INT64, synth.NUMERIC, 8, 8)] * 50)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["chunks", "product", "no_scratch"])
@pytest.mark.parametrize("with_coords", [False, True])
def test_gpu_batch_regions_by_lookup(oracle, case, with_coords):
    """Large mixed-schema batches take hash + separate lookups (hdx_kernels.hip
    case 212, hdx_regions.hip regions_by_lookup).  "chunks": debug variant 235
    (by lookup at any n, 64 MiB of scratch per chunk when no coordinates are
    wanted): 100 attributes -> 83 886 objects per chunk, so 200 003 objects are
    3 chunks, the last one ragged.  "product": the product library from its
    threshold (2^20 objects) on.  "no_scratch": debug variant 247, the same
    with the scratch allocation failing — the call falls back to the fused
    launch, which needs none."""
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import RegionTable, _lib
    dev = torch.device("cuda", 0)
    if case in ("chunks", "no_scratch"):
        rules, n, attrs3 = WIDE_MIXED, 200_003, [1, 2, 99]
    else:
        rules, n, attrs3 = WIDE_MIXED[:2] + WIDE_MIXED[:1], (1 << 20) + 4097, [1, 2, 0]
    types, blob, base, lens = synth.make_batch_host(rules, n, seed=77)
    assert hdx.hashing.kernel_for(types, n)[0] == 212
    want_coords, _ = oracle.hash_batch(types, blob, base, lens)
    specs = [([0],) + tuple(oracle.partition(1, 64)), (attrs3,) + tuple(oracle.partition(3, 64))]
    tables = [RegionTable(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 5) for at, lo, up in specs]
    variant = {"chunks": 235, "no_scratch": 247}.get(case)
    with _lib.debug_library(variant) if variant else contextlib.nullcontext():
        out = hdx.hash_batch_regions(types, torch.from_numpy(blob).to(dev),
                                     torch.from_numpy(base.view(np.int64)).to(dev),
                                     torch.from_numpy(lens.view(np.int32)).to(dev), tables, coords=with_coords)
        torch.cuda.synchronize()
    ids, coords = out if with_coords else (out, None)
    for k, (at, lo, up) in enumerate(specs):
        want = oracle.lookup_region(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 5, want_coords)
        assert np.array_equal(ids[k].cpu().numpy().view(np.uint64), want), k
    if with_coords:
        assert np.array_equal(coords.cpu().numpy().view(np.uint64), want_coords)
    for t in tables:
        t.close()


@pytest.mark.gpu
def test_gpu_regions_scratch_pool_across_calls_and_shutdown(oracle):
    """The regions scratch comes from the library's per-device memory pool
    (hdx_regions.hip region_pool): chunks reused call after call from the
    pool's cache, the cache trimmed by hdx_shutdown, and the next call after it
    allocating afresh — the same region ids every time (debug variant 235:
    three 64 MiB chunks per call)."""
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import RegionTable, _lib
    dev = torch.device("cuda", 0)
    n = 200_003
    types, blob, base, lens = synth.make_batch_host(WIDE_MIXED, n, seed=78)
    want_coords, _ = oracle.hash_batch(types, blob, base, lens)
    specs = [([0],) + tuple(oracle.partition(1, 64)), ([1, 2, 99],) + tuple(oracle.partition(3, 64))]
    ids_of = [np.arange(1, len(lo) + 1, dtype=np.uint64) * 3 for _, lo, _ in specs]
    want = [oracle.lookup_region(at, lo, up, ids_of[k], want_coords) for k, (at, lo, up) in enumerate(specs)]
    d = (torch.from_numpy(blob).to(dev), torch.from_numpy(base.view(np.int64)).to(dev),
         torch.from_numpy(lens.view(np.int32)).to(dev))
    with _lib.debug_library(235):
        for step in range(4):
            if step == 2:
                hdx.shutdown()  # trims the pool; the next call allocates again
            tables = [RegionTable(at, lo, up, ids_of[k]) for k, (at, lo, up) in enumerate(specs)]
            ids = hdx.hash_batch_regions(types, *d, tables)
            torch.cuda.synchronize()
            for k in range(len(specs)):
                assert np.array_equal(ids[k].cpu().numpy().view(np.uint64), want[k]), (step, k)
            for t in tables:
                t.close()


@pytest.mark.gpu
@pytest.mark.parametrize("form", list(range(100, 112)) + [217])
def test_gpu_batch_regions_every_fused_form(oracle, form):
    """The debug library's fused forms (hdx_kernels_dbg.hip launch_fused_debug:
    chunks per wave, sorted or not, tables in LDS or global memory, the
    per-lane or wave-uniform table loop) all give the oracle's region ids."""
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import RegionTable, _lib, synth
    dev = torch.device("cuda", 0)
    with _lib.debug_library(form):
        for cfg, n in [("cfg2", 1537), ("cfg3b", 777), ("mixed", 300), ("cfg1", 129)]:
            types, blob, base, lens = synth.make_batch_host(cfg, n, seed=form + n)
            want_coords, _ = oracle.hash_batch(types, blob, base, lens)
            A = len(types)
            specs = [([0],) + tuple(oracle.partition(1, 64))]
            if A >= 4:
                specs.append(([1, 2, 3],) + tuple(oracle.partition(3, 64)))
            tables = [RegionTable(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64)) for at, lo, up in specs]
            ids = hdx.hash_batch_regions(types, torch.from_numpy(np.ascontiguousarray(blob)).to(dev),
                                         torch.from_numpy(base.view(np.int64)).to(dev),
                                         torch.from_numpy(lens.view(np.int32)).to(dev), tables)
            torch.cuda.synchronize()
            for k, (at, lo, up) in enumerate(specs):
                want = oracle.lookup_region(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64), want_coords)
                assert np.array_equal(ids[k].cpu().numpy().view(np.uint64), want), (cfg, k)
            for t in tables:
                t.close()


@pytest.mark.gpu
def test_gpu_tables_used_on_another_device_get_a_replica(oracle):
    """A region table records the device it was created on; a call on another
    device (the device set's entry points run every device of the set) uses a
    replica of the table's host copy uploaded there on first use, never the
    creating device's memory.  One GPU here, so the table's device
    field (the first int of hdx_region_table_s, hdx_host.h) is rewritten to
    another ordinal: the fused and plain lookups then run on a replica and
    must give the same ids; the replica is freed with the table."""
    import ctypes

    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import regions, synth
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_device("cfg2", 1000, device=dev)
    lo, up = oracle.partition(1, 64)
    ids = np.arange(1, 65, dtype=np.uint64)
    t = regions.RegionTable([0], lo, up, ids)
    field = ctypes.c_int.from_address(t.handle.value)
    assert field.value == 0
    coords = hdx.hash_batch(types, blob, base, lens)
    want = oracle.lookup_region([0], lo, up, ids, coords.cpu().numpy().view(np.uint64))
    try:
        field.value = 5
        got1 = hdx.hash_batch_regions(types, blob, base, lens, [t])[0]
        got2 = regions.lookup_region(t, coords)
        torch.cuda.synchronize()
    finally:
        field.value = 0
    assert np.array_equal(got1.cpu().numpy().view(np.uint64), want)
    assert np.array_equal(got2.cpu().numpy().view(np.uint64), want)
    got3 = hdx.hash_batch_regions(types, blob, base, lens, [t])[0]
    torch.cuda.synchronize()
    assert np.array_equal(got3.cpu().numpy().view(np.uint64), want)
    t.close()


def _pack_keys(keys, dev):
    import torch
    lens = np.array([len(k) for k in keys], np.uint32)
    base = np.zeros(len(keys), np.uint64)
    base[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    blob = np.frombuffer(b"".join(keys) + b"\0" * 64, np.uint8)
    return (torch.from_numpy(blob.copy()).to(dev), torch.from_numpy(base.view(np.int64)).to(dev),
            torch.from_numpy(lens.view(np.int32)).to(dev))


def test_point_leader_oracle_semantics(oracle):
    """configuration.cc:440-454: first subspace-0 region, replicas[0].vsi,
    0 without replicas, abort without a region (the oracle flags it)."""
    h = [oracle.cityhash64(k) for k in (b"a", b"b", b"c")]
    lo = np.array([0, 0], np.uint64)
    up = np.array([U64MAX, U64MAX], np.uint64)
    got, ab = oracle.point_leader(9217, [b"a", b"b"], lo, up, [11, 12], [1, 1])
    assert list(got) == [11, 11] and not ab.any()  # the first region wins
    got, ab = oracle.point_leader(9217, [b"a"], lo, up, [11, 12], [0, 1])
    assert list(got) == [0] and not ab.any()  # no replicas: virtual_server_id()
    lo1 = np.array([h[0]], np.uint64)
    got, ab = oracle.point_leader(9217, [b"a", b"b", b"c"], lo1, lo1, [5], [1])
    assert got[0] == 5 and not ab[0] and (ab[1:] == [h[1] != h[0], h[2] != h[0]]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("key_type", [9217, 9218])
def test_gpu_point_leaders_match_oracle(oracle, key_type):
    """PointLeaders (one fused launch, two tables) == the oracle's restatement
    of point_leader for keys hitting every subspace-0 region of a 64-server
    key subspace, with a tenth of the regions replica-less."""
    import torch

    from hyperdex_amd import regions
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(key_type)
    if key_type == 9217:
        keys = [rng.integers(0, 256, int(rng.integers(0, 100)), dtype=np.uint8).tobytes() for _ in range(20000)]
    else:  # int64 keys spread over the whole ordered-encoding line
        keys = [int(x).to_bytes(8, "little", signed=True)
                for x in rng.integers(-2**63, 2**63 - 1, 20000, dtype=np.int64)]
    lo, up = oracle.partition(1, 64)
    vsi = rng.integers(1, 2**63, 64, dtype=np.uint64)
    has = rng.random(64) > 0.1
    pl = regions.PointLeaders(lo[:, 0], up[:, 0], vsi, has)
    try:
        leader, where = pl.leaders(key_type, *_pack_keys(keys, dev))
        torch.cuda.synchronize()
        want, aborted = oracle.point_leader(key_type, keys, lo[:, 0], up[:, 0], vsi, has)
        assert not aborted.any()
        assert np.array_equal(leader.cpu().numpy().view(np.uint64), want)
        assert len(np.unique(where.cpu().numpy())) == 64  # every region is hit
        assert (want == 0).sum() > 0  # replica-less regions answer virtual_server_id()
    finally:
        pl.close()


@pytest.mark.gpu
def test_gpu_point_leader_abort_is_reported(oracle):
    """A subspace-0 table with a hole: the keys in it are where the reference
    abort()s; PointLeaders raises, and without the check flags them 0."""
    import torch

    from hyperdex_amd import regions
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(7)
    keys = [rng.integers(0, 256, 24, dtype=np.uint8).tobytes() for _ in range(4000)]
    lo, up = oracle.partition(1, 16)
    keep = np.arange(16) != 5
    vsi = np.arange(100, 116, dtype=np.uint64)
    pl = regions.PointLeaders(lo[keep, 0], up[keep, 0], vsi[keep], np.ones(15, bool))
    try:
        packed = _pack_keys(keys, dev)
        with pytest.raises(regions.PointLeaderAbort):
            pl.leaders(9217, *packed)
        leader, where = pl.leaders(9217, *packed, check=False)
        torch.cuda.synchronize()
        want, aborted = oracle.point_leader(9217, keys, lo[keep, 0], up[keep, 0], vsi[keep], np.ones(15, bool))
        assert aborted.any()
        assert np.array_equal(where.cpu().numpy() == 0, aborted)
        assert np.array_equal(leader.cpu().numpy().view(np.uint64), want)
    finally:
        pl.close()
