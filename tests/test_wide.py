"""The reference's whole attribute domain (VERDICT r4 "do this" #3).

schema::attrs_sz is a u16 (common/schema.h:49), hash() loops over every
attribute (common/hash.cc:64-67) and encode_value writes up to 65535 of them
(daemon/datalayer_encodings.cc:145).  Every entry point — device batch, host
batch, device and host sweep, the regions forms — takes any attrs_sz up to
HDX_MAX_ATTRS = 65535: 129-256 attributes run the regroup kernel (44) or the
wide sweep, more than 256 the wide kernels of hdx_wide.hip.  GPU results are
compared with the oracle (oracle/hdx_oracle.c, no attribute cap) at A = 129,
200, 256, 257 and 1000 (and 4097 on the device batch)."""
import numpy as np
import pytest

from hyperdex_amd import _lib, synth
from hyperdex_amd import datatypes as dt

S, U, N = dt.HYPERDATATYPE_STRING, synth.UNIFORM, synth.NUMERIC


def wide_rules(A, seed):
    """A mix of every class: strings of every CityHash regime, int64, float,
    timestamps and non-hashable containers, key first."""
    rng = np.random.default_rng(seed)
    pool = [synth.Rule(S, U, 0, 16), synth.Rule(S, U, 0, 70), synth.Rule(S, U, 60, 200),
            synth.Rule(dt.HYPERDATATYPE_INT64, N, 8, 8), synth.Rule(dt.HYPERDATATYPE_FLOAT, N, 8, 8),
            synth.Rule(dt.HYPERDATATYPE_TIMESTAMP_DAY, N, 8, 8),
            synth.Rule(dt.HYPERDATATYPE_LIST_STRING, U, 0, 30)]
    return [synth.Rule(S, synth.FIXED, 24, 24)] + [pool[int(k)] for k in rng.integers(0, len(pool), A - 1)]


WIDTHS = [(129, 400), (200, 300), (256, 257), (257, 300), (1000, 130)]


def _dev_batch(torch, dev, blob, base, lens):
    return (torch.from_numpy(np.ascontiguousarray(blob) if len(blob) else np.zeros(1, np.uint8)).to(dev),
            torch.from_numpy(base.view(np.int64)).to(dev), torch.from_numpy(lens.view(np.int32)).to(dev))


def _tables(oracle, A, rng):
    """A key grid, a 3-attribute grid over high attribute indices and a scanned table of 300 random boxes."""
    from hyperdex_amd import RegionTable
    lo3, up3 = oracle.partition(3, 64)
    a = rng.integers(0, 2**64, size=(300, 2), dtype=np.uint64)
    b = rng.integers(0, 2**64, size=(300, 2), dtype=np.uint64)
    specs = [([0],) + tuple(oracle.partition(1, 64)), ([A - 1, A // 2, 1], lo3, up3),
             ([A - 2, 0], np.minimum(a, b), np.maximum(a, b))]
    return specs, [RegionTable(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 7) for at, lo, up in specs]


def _want_ids(oracle, specs, coords):
    return [oracle.lookup_region(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 7, coords)
            for at, lo, up in specs]


def test_schema_accepts_the_reference_domain():
    import hyperdex_amd as hdx
    assert _lib.HDX_MAX_ATTRS == 65535
    hdx.schema_check([S] * 65535)
    with pytest.raises(hdx.HdxError) as e:
        hdx.schema_check([S] * 65536)
    assert e.value.status == _lib.HDX_E_INVALID


def test_cpu_per_object_any_width(oracle):
    """hdx_hash_object (the C++ drop-in's path) at A = 1000 and 65535."""
    import hyperdex_amd as hdx
    pool = [S, dt.HYPERDATATYPE_INT64, dt.HYPERDATATYPE_FLOAT, dt.HYPERDATATYPE_TIMESTAMP_HOUR,
            dt.HYPERDATATYPE_MAP_STRING_STRING]
    for A in (1000, 65535):
        rng = np.random.default_rng(A)
        types = np.array([S] + [pool[int(k)] for k in rng.integers(0, len(pool), A - 1)], np.uint32)
        numeric = (types == dt.HYPERDATATYPE_INT64) | (types == dt.HYPERDATATYPE_FLOAT) | \
            (types == dt.HYPERDATATYPE_TIMESTAMP_HOUR)
        L = np.where(numeric, np.where(rng.random(A) < 0.05, 0, 8), rng.integers(0, 150, A)).astype(np.uint32)
        blob = rng.integers(0, 256, int(L.sum()), dtype=np.uint8)
        want, err = oracle.hash_batch(types, blob, np.zeros(1, np.uint64), L)
        assert err == 0
        offs = np.concatenate([[0], np.cumsum(L.astype(np.int64))])
        parts = [bytes(blob[offs[j]:offs[j + 1]]) for j in range(A)]
        assert hdx.hash_object(list(types), parts[0], parts[1:]) == [int(x) for x in want[0]]


@pytest.mark.gpu
@pytest.mark.parametrize("A,n", WIDTHS + [(4097, 9)])
def test_gpu_batch_any_width(oracle, A, n):
    """hdx_hash_batch_device: 44 up to 256 attributes, the wide kernel above."""
    import torch

    import hyperdex_amd as hdx
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_host(wide_rules(A, A + n), n, seed=A)
    want, err = oracle.hash_batch(types, blob, base, lens)
    assert err == 0
    assert hdx.hashing.kernel_for(types, n)[0] in ((44, 46) if A <= 256 else (300,))
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    got = hdx.hash_batch(types, *_dev_batch(torch, dev, blob, base, lens), status=status)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)
    assert int(status.item()) == 0


@pytest.mark.gpu
def test_gpu_wide_batch_bad_size_and_layouts(oracle):
    """The wide kernel on shuffled objects with gaps, and a mis-sized numeric
    (status bit, the other objects exact)."""
    import torch

    import hyperdex_amd as hdx
    dev = torch.device("cuda", 0)
    A, n = 300, 500
    types, blob, base, lens = synth.make_batch_host(wide_rules(A, 5), n, seed=5)
    rng = np.random.default_rng(5)
    perm = rng.permutation(n)
    L = lens.reshape(n, A)
    sizes = L.astype(np.uint64).sum(axis=1)
    gap = rng.integers(0, 9, n).astype(np.uint64)
    nbase = np.zeros(n, np.uint64)
    cur = 3
    out = np.zeros(int(sizes.sum() + gap.sum()) + 16, np.uint8)
    for i in perm:
        out[cur:cur + int(sizes[i])] = blob[int(base[i]):int(base[i] + sizes[i])]
        nbase[i] = cur
        cur += int(sizes[i] + gap[i])
    want, _ = oracle.hash_batch(types, out, nbase, lens)
    got = hdx.hash_batch(types, *_dev_batch(torch, dev, out, nbase, lens))
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)
    num = [j for j in range(A) if types[j] == dt.HYPERDATATYPE_INT64][0]
    bad = lens.copy()
    bad[7 * A + num] = 5  # object 7 now overlaps its neighbour's bytes: compare the others only
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    got = hdx.hash_batch(types, *_dev_batch(torch, dev, out, nbase, bad), status=status)
    torch.cuda.synchronize()
    assert int(status.item()) == 1 << _lib.HDX_E_BADSIZE
    g = got.cpu().numpy().view(np.uint64)
    assert g[7, num] == 0
    keep = np.arange(n) != 7
    assert np.array_equal(g[keep], want[keep])


@pytest.mark.gpu
@pytest.mark.parametrize("A,n", WIDTHS)
def test_gpu_host_batch_any_width(oracle, A, n):
    import hyperdex_amd as hdx
    types, blob, base, lens = synth.make_batch_host(wide_rules(A, A), n, seed=A + 1)
    want, _ = oracle.hash_batch(types, blob, base, lens)
    assert np.array_equal(hdx.hash_batch_host(types, blob, base, lens), want)


@pytest.mark.gpu
@pytest.mark.parametrize("A,n", WIDTHS)
def test_gpu_sweep_any_width(oracle, A, n):
    """hdx_hash_encoded_device and hdx_hash_encoded_host: the wide sweep above
    128 attributes, with corrupt values (zero coordinates, version 0,
    HDX_E_BADENC) among them."""
    import torch

    import hyperdex_amd as hdx
    from test_encoded import _corrupt, _to_dev
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_host(wide_rules(A, A + 2), n, seed=A + 2)
    enc = synth.encode_values_host(types, blob, base, lens, first_version=99)
    want, wver, bad = oracle.hash_encoded(types, *enc)
    assert not bad.any()
    versions = torch.zeros(n, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    got = hdx.hash_encoded(types, *_to_dev(torch, dev, enc), versions=versions, status=status)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)
    assert np.array_equal(versions.cpu().numpy().view(np.uint64), wver)
    assert int(status.item()) == 0
    c, v = hdx.hash_encoded_host(types, *enc, versions=True)
    assert np.array_equal(c, want) and np.array_equal(v, wver)
    enc2, cases = _corrupt(enc, np.random.default_rng(A))
    want2, wver2, bad2 = oracle.hash_encoded(types, *enc2)
    assert bad2.sum() == len(cases)
    status.zero_()
    got2 = hdx.hash_encoded(types, *_to_dev(torch, dev, enc2), versions=versions, status=status)
    torch.cuda.synchronize()
    assert np.array_equal(got2.cpu().numpy().view(np.uint64), want2)
    assert np.array_equal(versions.cpu().numpy().view(np.uint64), wver2)
    assert int(status.item()) == 1 << _lib.HDX_E_BADENC
    c2, v2, st, msg = hdx.hash_encoded_host_status(types, *enc2)
    assert st == _lib.HDX_E_BADENC and "decode" in msg
    assert np.array_equal(c2, want2) and np.array_equal(v2, wver2)


@pytest.mark.gpu
@pytest.mark.parametrize("A,n", WIDTHS)
def test_gpu_regions_any_width(oracle, A, n):
    """The regions entry points above 128 attributes (hash, then one lookup
    launch per table): device batch, host batch, device sweep, host sweep —
    with and without coordinates — against the oracle's lookup_region."""
    import torch

    import hyperdex_amd as hdx
    from test_encoded import _to_dev
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_host(wide_rules(A, A + 3), n, seed=A + 3)
    want_coords, _ = oracle.hash_batch(types, blob, base, lens)
    specs, tables = _tables(oracle, A, np.random.default_rng(A))
    wants = _want_ids(oracle, specs, want_coords)
    for with_coords in (False, True):
        out = hdx.hash_batch_regions(types, *_dev_batch(torch, dev, blob, base, lens), tables, coords=with_coords)
        torch.cuda.synchronize()
        ids = out[0] if with_coords else out
        for k in range(len(specs)):
            assert np.array_equal(ids[k].cpu().numpy().view(np.uint64), wants[k]), (with_coords, k)
        if with_coords:
            assert np.array_equal(out[1].cpu().numpy().view(np.uint64), want_coords)
        hout = hdx.hash_batch_regions_host(types, blob, base, lens, tables, coords=with_coords)
        hids = hout[0] if with_coords else hout
        assert all(np.array_equal(hids[k], wants[k]) for k in range(len(specs)))
        if with_coords:
            assert np.array_equal(hout[1], want_coords)
    enc = synth.encode_values_host(types, blob, base, lens)
    for with_coords in (False, True):
        out = hdx.hash_encoded_regions(types, *_to_dev(torch, dev, enc), tables, coords=with_coords)
        torch.cuda.synchronize()
        ids = out[0] if with_coords else out
        assert all(np.array_equal(ids[k].cpu().numpy().view(np.uint64), wants[k]) for k in range(len(specs)))
    c, v, st, msg, hids = hdx.hash_encoded_host_status(types, *enc, tables=tables)
    assert st == _lib.HDX_OK, msg
    assert np.array_equal(c, want_coords)
    assert all(np.array_equal(hids[k], wants[k]) for k in range(len(specs)))
    for t in tables:
        t.close()


def _ring_rules(A, seed):
    """Attributes of 0 bytes up to 9 KiB among short ones: prefixes at every
    place of the wide sweep's LDS ring (across a chunk's end and the ring's
    wrap) and jumps past the prefetched chunk (one attribute longer than a
    chunk, or than the whole ring)."""
    rng = np.random.default_rng(seed)
    pool = [synth.Rule(S, U, 0, 40), synth.Rule(S, U, 0, 300), synth.Rule(S, U, 1000, 5000),
            synth.Rule(S, U, 4000, 9300), synth.Rule(dt.HYPERDATATYPE_INT64, N, 8, 8),
            synth.Rule(dt.HYPERDATATYPE_FLOAT, N, 8, 8)]
    p = np.array([0.4, 0.3, 0.05, 0.03, 0.11, 0.11])
    return [synth.Rule(S, U, 0, 100)] + [pool[int(k)] for k in rng.choice(len(pool), A - 1, p=p)]


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [-1, 304, 305, 306, 309, 310, 311, 312])
def test_gpu_sweep_stream_ring(oracle, variant):
    """The wide sweep on values of 10 bytes to ~100 KB at every 16-byte
    alignment, with corrupt ones: the product (the lane-per-object walk, its
    descriptors stored 16 at a time, then the hash) and the debug forms — 304 /
    305 / 306 a wave per object streaming the value through a two-chunk LDS
    ring of 4 / 2 / 8 KiB chunks (prefixes across a chunk's end and the ring's
    wrap, jumps past the prefetched chunk), 309 / 310 the walk storing 1 / 8
    descriptors at a time, 311 the hash class-sorted, 312 one launch with a
    lane per object walking and hashing."""
    import contextlib

    import torch

    import hyperdex_amd as hdx
    from test_encoded import _corrupt, _to_dev
    dev = torch.device("cuda", 0)
    with _lib.debug_library(variant) if variant >= 0 else contextlib.nullcontext():
        for A, n in ((130, 120), (700, 24)):
            types, blob, base, lens = synth.make_batch_host(_ring_rules(A, A + 5), n, seed=A + 6)
            enc = synth.encode_values_host(types, blob, base, lens, first_version=17)
            enc, cases = _corrupt(enc, np.random.default_rng(A)) if n >= 100 else (enc, {})
            want, wver, bad = oracle.hash_encoded(types, *enc)
            assert bad.sum() == len(cases)
            versions = torch.zeros(n, dtype=torch.int64, device=dev)
            status = torch.zeros(1, dtype=torch.int32, device=dev)
            got = hdx.hash_encoded(types, *_to_dev(torch, dev, enc), versions=versions, status=status)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy().view(np.uint64), want), (A, n)
            assert np.array_equal(versions.cpu().numpy().view(np.uint64), wver), (A, n)
            assert int(status.item()) == (1 << _lib.HDX_E_BADENC if cases else 0)
