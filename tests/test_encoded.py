"""Reindex sweep over stored objects (config 5): decode_value
(daemon/datalayer_encodings.cc:168-217) + hash, GPU vs oracle."""
import numpy as np
import pytest

from hyperdex_amd import _lib, synth


def test_oracle_decodes_what_encode_wrote(oracle):
    types, blob, base, lens = synth.make_batch_host("cfg3b", 300, seed=5)
    enc = synth.encode_values_host(types, blob, base, lens, first_version=1000)
    coords, versions, bad = oracle.hash_encoded(types, *enc)
    want, _ = oracle.hash_batch(types, blob, base, lens)
    assert not bad.any()
    assert np.array_equal(coords, want)
    assert np.array_equal(versions, 1000 + np.arange(300, dtype=np.uint64))


def _corrupt(enc, rng):
    """Truncations, bad counts, overrunning lengths, tiny and empty values."""
    keys, key_off, key_len, vals, val_off, val_len = [np.array(x) for x in enc]
    n = len(val_off)
    cases = {}
    for i in rng.choice(n, 40, replace=False):
        kind = len(cases) % 5
        o, L = int(val_off[i]), int(val_len[i])
        if kind == 0:
            val_len[i] = rng.integers(0, 10)          # shorter than the header
        elif kind == 1:
            vals[o + 9] ^= 1                           # count != A-1
        elif kind == 2:
            val_len[i] = L - rng.integers(1, 5)        # last attribute runs past the end
        elif kind == 3:
            vals[o + 10:o + 14] = [0xff, 0xff, 0xff, 0xf0]  # first length overruns
        else:
            val_len[i] = 10 + 2                        # truncated length prefix
        cases[int(i)] = kind
    return (keys, key_off, key_len, vals, val_off, val_len), cases


def test_oracle_rejects_corrupt_values(oracle):
    types, blob, base, lens = synth.make_batch_host("cfg3b", 200, seed=6)
    enc, cases = _corrupt(synth.encode_values_host(types, blob, base, lens), np.random.default_rng(1))
    coords, versions, bad = oracle.hash_encoded(types, *enc)
    assert set(np.nonzero(bad)[0]) == set(cases)
    assert (coords[bad] == 0).all() and (versions[bad] == 0).all()


def _to_dev(torch, dev, arrs):
    out = []
    for a in arrs:
        a = np.ascontiguousarray(a)
        if a.dtype == np.uint64:
            a = a.view(np.int64)
        elif a.dtype == np.uint32:
            a = a.view(np.int32)
        if a.size == 0:
            a = np.zeros(1, a.dtype)
        out.append(torch.from_numpy(a.copy()).to(dev))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,n", [("cfg3b", 3000), ("cfg2", 5000), ("mixed", 3000), ("cfg1", 2000),
                                   ("wide", 300)])
def test_gpu_encoded_matches_oracle(oracle, cfg, n):
    import torch

    import hyperdex_amd as hdx
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_host(cfg, n, seed=n + 3)
    enc = synth.encode_values_host(types, blob, base, lens, first_version=77)
    want, wver, _ = oracle.hash_encoded(types, *enc)
    d = _to_dev(torch, dev, enc)
    versions = torch.zeros(n, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    got = hdx.hash_encoded(types, *d, versions=versions, status=status)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)
    assert np.array_equal(versions.cpu().numpy().view(np.uint64), wver)
    assert int(status.item()) == 0


@pytest.mark.gpu
def test_gpu_encoded_corrupt_values(oracle):
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import _lib
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_host("cfg3b", 1000, seed=9)
    enc, cases = _corrupt(synth.encode_values_host(types, blob, base, lens), np.random.default_rng(2))
    want, wver, bad = oracle.hash_encoded(types, *enc)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    versions = torch.zeros(1000, dtype=torch.int64, device=dev)
    got = hdx.hash_encoded(types, *_to_dev(torch, dev, enc), versions=versions, status=status)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)
    assert np.array_equal(versions.cpu().numpy().view(np.uint64), wver)
    assert int(status.item()) == 1 << _lib.HDX_E_BADENC


@pytest.mark.gpu
def test_gpu_encoded_device_generator(oracle):
    """make_encoded_device (HBM encoder) == host encoder, and the sweep is exact."""
    import torch

    import hyperdex_amd as hdx
    dev = torch.device("cuda", 0)
    types, keys, key_off, key_len, vals, val_off, val_len = synth.make_encoded_device("cfg3b", 4000, device=dev)
    h = synth.encode_values_host(*synth.make_batch_host("cfg3b", 4000))
    assert np.array_equal(vals.cpu().numpy()[:len(h[3])], h[3])
    assert np.array_equal(val_off.cpu().numpy().view(np.uint64), h[4])
    got = hdx.hash_encoded(types, keys, key_off, key_len, vals, val_off, val_len)
    torch.cuda.synchronize()
    want, _, _ = oracle.hash_encoded(types, *h)
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)


@pytest.mark.gpu
@pytest.mark.parametrize("A,n", [(33, 66), (5, 104), (2, 100), (17, 70), (65, 130), (70, 130), (128, 65)])
def test_gpu_encoded_partial_last_pass(oracle, A, n):
    """Last wave with few objects: its final pass has most lanes past the batch
    end while the active lanes need other objects' bases and other positions'
    codes (regression: cross-lane reads from inactive lanes return 0)."""
    import torch

    import hyperdex_amd as hdx
    rules = [synth.Rule(9217, synth.UNIFORM, 0, 130)] * (A - 2) + [synth._n(9218), synth._n(9219)]
    types, blob, base, lens = synth.make_batch_host(rules[:A], n, seed=A * 1000 + n)
    enc = synth.encode_values_host(types, blob, base, lens)
    want, _, _ = oracle.hash_encoded(types, *enc)
    got = hdx.hash_encoded(types, *_to_dev(torch, torch.device("cuda", 0), enc))
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)


def _scatter(enc, rng):
    """The same objects with their keys and values moved to a shuffled order
    with gaps between them (no group of objects is a contiguous run)."""
    keys, key_off, key_len, vals, val_off, val_len = [np.array(x) for x in enc]

    def move(buf, off, ln):
        n = len(off)
        order = rng.permutation(n)
        out = np.zeros(int(ln.astype(np.int64).sum()) + 41 * n + 16, np.uint8)
        new_off = np.zeros(n, np.uint64)
        cur = int(rng.integers(0, 16))
        for i in order:
            L = int(ln[i])
            out[cur:cur + L] = buf[int(off[i]):int(off[i]) + L]
            new_off[i] = cur
            cur += L + int(rng.integers(0, 41))
        return out[:max(cur, 1)], new_off

    keys2, key_off2 = move(keys, key_off, key_len)
    vals2, val_off2 = move(vals, val_off, val_len)
    return keys2, key_off2, key_len, vals2, val_off2, val_len


def test_oracle_scattered_layout(oracle):
    types, blob, base, lens = synth.make_batch_host("cfg3b", 120, seed=4)
    enc = synth.encode_values_host(types, blob, base, lens)
    want = oracle.hash_encoded(types, *enc)
    got = oracle.hash_encoded(types, *_scatter(enc, np.random.default_rng(3)))
    assert all(np.array_equal(x, y) for x, y in zip(got, want))


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [-1, 43, 47, 49, 301, 170, 171, 173, 230, 232, 236, 239, 242, 243, 244, 245, 246, 250, 251, 253, 254, 255])
def test_gpu_encoded_scattered_layout(oracle, variant):
    """Objects whose keys and values lie in shuffled order with gaps hash
    exactly as the packed layout does."""
    import torch

    import hyperdex_amd as hdx
    dev = torch.device("cuda", 0)
    with _lib.debug_library(variant):
        for cfg, n in (("cfg3b", 700), ("mixed", 300), ("cfg2", 129)):
            types, blob, base, lens = synth.make_batch_host(cfg, n, seed=n + 11)
            enc = synth.encode_values_host(types, blob, base, lens, first_version=9)
            want, wver, _ = oracle.hash_encoded(types, *enc)
            enc2 = _scatter(enc, np.random.default_rng(n))
            versions = torch.zeros(n, dtype=torch.int64, device=dev)
            got = hdx.hash_encoded(types, *_to_dev(torch, dev, enc2), versions=versions)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy().view(np.uint64), want), (cfg, n)
            assert np.array_equal(versions.cpu().numpy().view(np.uint64), wver), (cfg, n)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [-1, 33, 43, 47, 48, 49, 301, 170, 171, 172, 173, 174, 230, 231, 232, 236, 239, 242, 243, 244, 245, 246, 250, 251, 253, 254, 255, 256, 257, 258, 259, 270, 271, 272, 273, 277, 293, 298])
def test_gpu_encoded_every_variant(oracle, variant):
    """Every stored-object sweep kernel (hdx_encoded.hip; 33 adds the line
    touch) is bit-exact on every config, on corrupt values, on ragged object
    counts and on large values (wide, keyonly_long)."""
    import torch

    import hyperdex_amd as hdx
    dev = torch.device("cuda", 0)
    with _lib.debug_library(variant):
        cases = [("cfg3b", 1001), ("cfg2", 997), ("mixed", 500), ("cfg1", 33), ("wide", 61),
                 ("keyonly_long", 40), ("cfg3b", 1), ("cfg3b", 15), ("cfg3b", 16)]
        for cfg, n in cases:
            types, blob, base, lens = synth.make_batch_host(cfg, n, seed=n * 7 + 1)
            enc = synth.encode_values_host(types, blob, base, lens, first_version=5)
            if cfg == "cfg3b" and n > 100:
                enc, _ = _corrupt(enc, np.random.default_rng(variant + 10))
            want, wver, _ = oracle.hash_encoded(types, *enc)
            versions = torch.zeros(n, dtype=torch.int64, device=dev)
            got = hdx.hash_encoded(types, *_to_dev(torch, dev, enc), versions=versions)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy().view(np.uint64), want), (cfg, n)
            assert np.array_equal(versions.cpu().numpy().view(np.uint64), wver), (cfg, n)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [-1, 301, 170, 171, 173, 174, 230, 232, 236, 239, 242, 243, 244, 245, 246, 250, 251, 253, 254, 255])
def test_gpu_encoded_bad_numeric_size(oracle, variant):
    """A stored int64 / float / timestamp value of neither 0 nor 8 bytes (the
    reference asserts, datatype_int64.cc:233): its coordinate is 0 and status
    gets HDX_E_BADSIZE; every other coordinate is the oracle's.  Values with
    just enough room for the prefix (no speculative 8-byte read past them)."""
    import struct

    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import _lib, datatypes as dt
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(variant + 100)
    types = [dt.HYPERDATATYPE_STRING, dt.HYPERDATATYPE_INT64, dt.HYPERDATATYPE_STRING,
             dt.HYPERDATATYPE_FLOAT, dt.TIMESTAMPS[2], dt.HYPERDATATYPE_LIST_STRING]
    n = 300
    keys, vals, want = [], [], np.zeros((n, len(types)), np.uint64)
    for i in range(n):
        key = rng.bytes(int(rng.integers(0, 80)))
        attrs = [rng.bytes(8) if rng.random() < 0.9 else b"", rng.bytes(int(rng.integers(0, 150))),
                 rng.bytes(8), rng.bytes(8) if rng.random() < 0.8 else b"", rng.bytes(int(rng.integers(0, 30)))]
        badk = int(rng.integers(0, 3)) if i % 7 == 3 else -1  # one of the numerics mis-sized
        if badk >= 0:
            attrs[(0, 2, 3)[badk]] = rng.bytes(int(rng.choice([1, 4, 7, 9, 16])))
        keys.append(key)
        vals.append(struct.pack(">QH", i, len(attrs)) + b"".join(struct.pack(">I", len(x)) + x for x in attrs))
        want[i, 0] = oracle.hash_value(types[0], key)[0]
        for k, x in enumerate(attrs):
            h, err = oracle.hash_value(types[k + 1], x)
            want[i, k + 1] = 0 if err else h
    key_len = np.array([len(k) for k in keys], np.uint32)
    val_len = np.array([len(v) for v in vals], np.uint32)
    key_off = np.concatenate([[0], np.cumsum(key_len)[:-1]]).astype(np.uint64)
    val_off = np.concatenate([[0], np.cumsum(val_len)[:-1]]).astype(np.uint64)
    enc = (np.frombuffer(b"".join(keys) + b"\0", np.uint8), key_off, key_len,
           np.frombuffer(b"".join(vals), np.uint8), val_off, val_len)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    with _lib.debug_library(variant):
        got = hdx.hash_encoded(types, *_to_dev(torch, dev, enc), status=status)
        torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)
    assert int(status.item()) == 1 << _lib.HDX_E_BADSIZE


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [-1, 233, 234])
@pytest.mark.parametrize("with_coords", [False, True])
def test_gpu_encoded_regions_fused(oracle, with_coords, variant):
    """hdx_hash_encoded_regions_device = the sweep's coordinates looked up in
    every table (an indexed 64-region key grid, an indexed 3-attribute grid,
    and a 300-region table that is scanned), corrupt values included; the
    product (the wave-staged sweep + separate lookups), the wave-staged sweep
    with the lookup fused (233) and the gather sweep's fused form (234)."""
    if variant >= 0:
        with _lib.debug_library(variant):
            _encoded_regions_fused(oracle, with_coords)
    else:
        _encoded_regions_fused(oracle, with_coords)


def _encoded_regions_fused(oracle, with_coords):
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import RegionTable
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_host("cfg3b", 3001, seed=31)
    enc = synth.encode_values_host(types, blob, base, lens, first_version=9)
    enc, _ = _corrupt(enc, np.random.default_rng(4))
    want_coords, _, _ = oracle.hash_encoded(types, *enc)
    rng = np.random.default_rng(5)
    lo1, up1 = oracle.partition(1, 64)
    lo3, up3 = oracle.partition(3, 64)
    a = rng.integers(0, 2**64, size=(300, 2), dtype=np.uint64)
    b = rng.integers(0, 2**64, size=(300, 2), dtype=np.uint64)
    specs = [([0], lo1, up1), ([1, 2, 3], lo3, up3), ([16, 5], np.minimum(a, b), np.maximum(a, b))]
    tables = [RegionTable(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 7) for at, lo, up in specs]
    out = hdx.hash_encoded_regions(types, *_to_dev(torch, dev, enc), tables, coords=with_coords)
    torch.cuda.synchronize()
    ids, coords = out if with_coords else (out, None)
    for k, (at, lo, up) in enumerate(specs):
        want = oracle.lookup_region(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 7, want_coords)
        assert np.array_equal(ids[k].cpu().numpy().view(np.uint64), want), k
    if with_coords:
        assert np.array_equal(coords.cpu().numpy().view(np.uint64), want_coords)
    for t in tables:
        t.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["chunks", "product", "no_scratch"])
@pytest.mark.parametrize("with_coords", [False, True])
def test_gpu_encoded_regions_by_lookup(oracle, case, with_coords):
    """The product's regions sweep from 2^20 objects on is the wave-staged
    sweep + separate lookups (hdx_regions.hip regions_by_lookup).  "chunks":
    debug variant 235 (by lookup at any n, 64 MiB of scratch per chunk when no
    coordinates are wanted): 100 attributes -> 83 886 objects per chunk, so
    200 003 stored objects are 3 chunks, the last one ragged.  "product": the
    product library past its threshold.  Versions and the status word follow
    the chunks."""
    import contextlib

    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import RegionTable
    dev = torch.device("cuda", 0)
    rules = [synth.Rule(synth.dt.HYPERDATATYPE_STRING, synth.UNIFORM, 0, 40),
             synth.Rule(synth.dt.HYPERDATATYPE_INT64, synth.NUMERIC, 8, 8)] * 50
    if case in ("chunks", "no_scratch"):
        n, attrs3 = 200_003, [1, 2, 99]
    else:
        rules, n, attrs3 = rules[:2] + rules[:1], (1 << 20) + 4097, [1, 2, 0]
    types, blob, base, lens = synth.make_batch_host(rules, n, seed=78)
    enc = synth.encode_values_host(types, blob, base, lens, first_version=3)
    want_coords, want_versions, _ = oracle.hash_encoded(types, *enc)
    specs = [([0],) + tuple(oracle.partition(1, 64)), (attrs3,) + tuple(oracle.partition(3, 64))]
    tables = [RegionTable(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 11) for at, lo, up in specs]
    versions = torch.empty(n, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    variant = {"chunks": 235, "no_scratch": 247}.get(case)
    with _lib.debug_library(variant) if variant else contextlib.nullcontext():
        out = hdx.hash_encoded_regions(types, *_to_dev(torch, dev, enc), tables, coords=with_coords,
                                       versions=versions, status=status)
        torch.cuda.synchronize()
    ids, coords = out if with_coords else (out, None)
    for k, (at, lo, up) in enumerate(specs):
        want = oracle.lookup_region(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 11, want_coords)
        assert np.array_equal(ids[k].cpu().numpy().view(np.uint64), want), k
    if with_coords:
        assert np.array_equal(coords.cpu().numpy().view(np.uint64), want_coords)
    assert np.array_equal(versions.cpu().numpy().view(np.uint64), want_versions)
    assert int(status.item()) == 0
    for t in tables:
        t.close()


# ---- records [key][value] back to back (a LevelDB block's adjacency) ----------

def test_oracle_records_layout(oracle):
    """encode_records_host: the same objects as one store of records decode
    and hash to the packed batch's coordinates."""
    types, blob, base, lens = synth.make_batch_host("cfg3b", 200, seed=51)
    rec = synth.encode_store_host(types, blob, base, lens, first_version=5)
    coords, versions, bad = oracle.hash_encoded(types, *rec)
    want, _ = oracle.hash_batch(types, blob, base, lens)
    assert not bad.any() and np.array_equal(coords, want)
    assert np.array_equal(versions, 5 + np.arange(200, dtype=np.uint64))


def _records_with_gaps(rec, rng):
    """Move a few records apart (gaps in the store): the groups holding them
    are no longer one run and take the key / value paths instead."""
    store, key_off, key_len, _, val_off, val_len = [np.array(x) for x in rec]
    n = len(key_off)
    shift = np.zeros(n, np.uint64)
    for i in sorted(rng.choice(n, max(1, n // 50), replace=False)):
        shift[i:] += np.uint64(int(rng.integers(1, 40)))
    out = np.zeros(len(store) + int(shift[-1]) + 64, np.uint8)
    for i in range(n):
        r, k, v = int(key_off[i]), int(key_len[i]), int(val_len[i])
        out[r + int(shift[i]):r + int(shift[i]) + k + v] = store[r:r + k + v]
    return out, key_off + shift, key_len, out, val_off + shift, val_len


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [-1, 250, 251, 253, 254, 255])
@pytest.mark.parametrize("case", ["packed", "gaps", "corrupt"])
def test_gpu_encoded_records(oracle, case, variant):
    """The sweep on the records layout: a group whose records are back to back
    is one span (keys and values read from it); gaps between records and
    corrupt values keep the reference's results; 250 = the product without the
    record span (round 3's key / value paths) on the same store."""
    import contextlib

    import torch

    import hyperdex_amd as hdx
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_host("cfg3b", 3001, seed=52)
    rec = synth.encode_store_host(types, blob, base, lens, first_version=11)
    rng = np.random.default_rng(53)
    if case == "gaps":
        rec = _records_with_gaps(rec, rng)
    elif case == "corrupt":
        enc, _ = _corrupt(rec, rng)
        rec = (enc[3],) + enc[1:3] + (enc[3],) + enc[4:]  # the corrupted store is both keys and values
    want, wver, _ = oracle.hash_encoded(types, *rec)
    d = _to_dev(torch, dev, rec)
    d[3] = d[0]  # one store on the device too
    versions = torch.zeros(len(rec[1]), dtype=torch.int64, device=dev)
    with _lib.debug_library(variant) if variant >= 0 else contextlib.nullcontext():
        got = hdx.hash_encoded(types, *d, versions=versions)
        torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), want)
    assert np.array_equal(versions.cpu().numpy().view(np.uint64), wver)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["keycol", "records"])
def test_gpu_encoded_store_device_generator(oracle, layout):
    """make_encoded_device(layout=...) writes exactly the host encoding, and
    the sweep over it (keys as one span, or records as one span) matches the
    oracle."""
    import torch

    import hyperdex_amd as hdx
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_host("cfg3b", 1500, seed=54, first=777)
    want = synth.encode_store_host(types, blob, base, lens, first_version=777, layout=layout)
    got = synth.make_encoded_device("cfg3b", 1500, seed=54, first=777, device=dev, layout=layout)
    assert np.array_equal(got[1].cpu().numpy()[:len(want[0])], want[0])
    assert np.array_equal(got[4].cpu().numpy()[:len(want[3])], want[3])
    for g, w in zip(got[2:4] + got[5:], want[1:3] + want[4:]):
        assert np.array_equal(g.cpu().numpy().view(w.dtype), w)
    coords, _, _ = oracle.hash_encoded(types, *want)
    c = hdx.hash_encoded(types, *got[1:])
    torch.cuda.synchronize()
    assert np.array_equal(c.cpu().numpy().view(np.uint64), coords)
