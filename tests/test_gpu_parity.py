"""GPU parity: the gfx950 kernels (through the C-ABI) vs the CPU oracle.

Bit-exact equality on every coordinate: integer/byte work has no tolerance.
Inputs: the reference KAT, the SURVEY §8c reference-produced values, seeded
synthetic batches of every config at oracle-friendly sizes, edge cases (empty
and ragged batches, wave boundaries, attribute-count extremes, gaps and
shuffled object order, unaligned strings), and a full BASELINE-size batch
checked by sampling + determinism.
"""
import json
import os
import struct

import numpy as np
import pytest

import hyperdex_amd as hdx
from hyperdex_amd import _lib, datatypes as dt, synth
from kat_data import kat_array

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available()
    return torch, torch.device("cuda", 0)


def to_dev(torch, dev, blob, base, lens):
    b = torch.from_numpy(np.ascontiguousarray(blob).view(np.uint8).copy()).to(dev)
    o = torch.from_numpy(np.ascontiguousarray(base, np.uint64).view(np.int64).copy()).to(dev)
    L = torch.from_numpy(np.ascontiguousarray(lens, np.uint32).view(np.int32).copy()).to(dev)
    return b, o, L


def gpu_hash(torch, dev, types, blob, base, lens, status=None):
    if len(blob) == 0:
        blob = np.zeros(1, np.uint8)
    b, o, L = to_dev(torch, dev, blob, base, lens)
    c = hdx.hash_batch(types, b, o, L, status=status)
    torch.cuda.synchronize()
    return c.cpu().numpy().view(np.uint64)


def check_batch(oracle, torch, dev, types, blob, base, lens):
    want, err = oracle.hash_batch(types, blob, base, lens)
    assert err == 0
    got = gpu_hash(torch, dev, types, blob, base, lens)
    bad = np.argwhere(got != want)
    assert bad.size == 0, "first mismatch at (obj, attr) %s: got %x want %x" % (
        tuple(bad[0]), got[tuple(bad[0])], want[tuple(bad[0])])
    return got


def test_kat_on_gpu(oracle, torch_dev):
    """All 300 reference CityHash64 vectors hashed in one device batch (A=1)."""
    torch, dev = torch_dev
    kat = json.load(open(os.path.join(GOLD, "cityhash64_kat.json")))["cases"]
    data = kat_array()
    base = np.array([c["offset"] for c in kat], np.uint64)
    lens = np.array([c["len"] for c in kat], np.uint32)
    got = gpu_hash(torch, dev, [dt.HYPERDATATYPE_STRING], data, base, lens)[:, 0]
    want = np.array([int(c["cityhash64"], 16) for c in kat], np.uint64)
    assert np.array_equal(got, want), np.nonzero(got != want)


def _enc(kind, value):
    if kind == "empty":
        return b""
    if kind == "bytes":
        return value.encode()
    if kind == "int64":
        return struct.pack("<q", value)
    return struct.pack("<Q", int(value, 16))


def test_reference_values_per_object_api(torch_dev):
    """hash(type, slice) and hash(schema, key, value, hs) through the C-ABI."""
    rv = json.load(open(os.path.join(GOLD, "reference_values.json")))
    for s in rv["scalars"]:
        assert hdx.hash(s["type"], _enc(s["kind"], s["value"])) == int(s["hash"], 16), s
    for o in rv["objects"]:
        sc = dt.Schema.of(*o["types"])
        hs = hdx.hash_object(sc, o["key"].encode(), [_enc(v["kind"], v["value"]) for v in o["values"]])
        assert ["%016x" % h for h in hs] == o["hashes"]
        assert hdx.hash_key(sc, o["key"].encode()) == int(o["hashes"][0], 16)


@pytest.mark.parametrize("cfg,n", [("cfg1", 5000), ("cfg2", 5000), ("cfg3a", 3000), ("cfg3b", 4000),
                                   ("mixed", 6000), ("wide", 500), ("keyonly_long", 700)])
def test_configs_match_oracle(oracle, torch_dev, cfg, n):
    torch, dev = torch_dev
    types, blob, base, lens = synth.make_batch_host(cfg, n, seed=synth.SEED + n)
    check_batch(oracle, torch, dev, types, blob, base, lens)


@pytest.mark.parametrize("n", [0, 1, 2, 63, 64, 65, 127, 129, 1000])
def test_ragged_object_counts(oracle, torch_dev, n):
    torch, dev = torch_dev
    types, blob, base, lens = synth.make_batch_host("mixed", n, seed=1000 + n)
    if n == 0:
        b, o, L = to_dev(torch, dev, np.zeros(1, np.uint8), np.zeros(0, np.uint64),
                         np.zeros(0, np.uint32))
        c = hdx.hash_batch(types, b, o, L)
        assert c.shape == (0, len(types))
        return
    check_batch(oracle, torch, dev, types, blob, base, lens)


@pytest.mark.parametrize("A", [1, 2, 3, 5, 31, 32, 33, 63, 64, 65, 100, 128, 255])
def test_attribute_counts(oracle, torch_dev, A):
    torch, dev = torch_dev
    rules = [synth.Rule(dt.HYPERDATATYPE_STRING, synth.UNIFORM, 0, 80)] * A
    types, blob, base, lens = synth.make_batch_host(rules, 150, seed=77 + A)
    check_batch(oracle, torch, dev, types, blob, base, lens)


@pytest.mark.parametrize("A", [2, 3, 17, 63, 64, 65, 100, 128, 129, 200])
def test_mixed_attribute_counts(oracle, torch_dev, A):
    """Mixed string / int64 / float schemas go through the product's
    wave-staged kernel up to 128 attributes (one object per wave at 65..128:
    objects straddle its passes), the gather kernel above."""
    torch, dev = torch_dev
    kinds = [synth.Rule(dt.HYPERDATATYPE_STRING, synth.UNIFORM, 0, 150),
             synth.Rule(dt.HYPERDATATYPE_INT64, synth.NUMERIC, 8, 8),
             synth.Rule(dt.HYPERDATATYPE_FLOAT, synth.NUMERIC, 8, 8)]
    rules = [kinds[j % 3] for j in range(A)]
    types, blob, base, lens = synth.make_batch_host(rules, 301, seed=555 + A)
    check_batch(oracle, torch, dev, types, blob, base, lens)


def test_every_string_length_and_alignment(oracle, torch_dev):
    """Lengths 0..520 at every byte alignment 0..15 (all CityHash regimes and
    1..8 iterations of the 64-byte loop)."""
    torch, dev = torch_dev
    rng = np.random.default_rng(5)
    lens = np.repeat(np.arange(521, dtype=np.uint32), 16)
    align = np.tile(np.arange(16, dtype=np.uint64), 521)
    stride = 544
    base = np.arange(len(lens), dtype=np.uint64) * stride + align
    blob = rng.integers(0, 256, int(base[-1]) + stride, dtype=np.uint8)
    check_batch(oracle, torch, dev, [dt.HYPERDATATYPE_STRING], blob, base, lens)


def test_gaps_and_shuffled_objects(oracle, torch_dev):
    torch, dev = torch_dev
    types, blob, base, lens = synth.make_batch_host("cfg3b", 3000, seed=99)
    n, A = len(base), len(types)
    rng = np.random.default_rng(3)
    perm = rng.permutation(n)
    sizes = lens.reshape(n, A).astype(np.uint64).sum(axis=1)
    gaps = rng.integers(0, 37, n).astype(np.uint64)
    new_base = np.zeros(n, np.uint64)
    pos = np.uint64(5)
    out = np.zeros(int(sizes.sum() + gaps.sum()) + 64, np.uint8)
    for k in perm:  # write objects in shuffled order with random gaps
        pos += gaps[k]
        new_base[k] = pos
        out[int(pos):int(pos + sizes[k])] = blob[int(base[k]):int(base[k] + sizes[k])]
        pos += sizes[k]
    got = check_batch(oracle, torch, dev, types, out, new_base, lens)
    want, _ = oracle.hash_batch(types, blob, base, lens)
    assert np.array_equal(got, want)


def test_float_and_int_specials(oracle, torch_dev):
    torch, dev = torch_dev
    vals = [0, 1 << 63, 0x7ff0000000000000, 0xfff0000000000000, 0x7ff8000000000000,
            0xfff8000000000001, 0x7ff0000000000001, 0xfff0000000000001, 1, (1 << 63) | 1,
            0x000fffffffffffff, 0x800fffffffffffff, 0x0010000000000000, 0x8010000000000000,
            0x7fefffffffffffff, 0xffefffffffffffff, 0x3ff0000000000000, 0xbff0000000000000,
            0x7fffffffffffffff, 0xffffffffffffffff]
    types = [dt.HYPERDATATYPE_FLOAT, dt.HYPERDATATYPE_INT64] + list(dt.TIMESTAMPS)
    A = len(types)
    blob = np.frombuffer(b"".join(struct.pack("<Q", v) for v in vals for _ in range(A)), np.uint8)
    base = np.arange(len(vals), dtype=np.uint64) * (8 * A)
    lens = np.full(len(vals) * A, 8, np.uint32)
    check_batch(oracle, torch, dev, types, blob, base, lens)


def test_timestamps_random(oracle, torch_dev):
    torch, dev = torch_dev
    rng = np.random.default_rng(11)
    n = 20000
    ts = np.concatenate([rng.integers(-2**63, 2**63 - 1, n // 2, dtype=np.int64),
                         rng.integers(0, 2**53, n // 2, dtype=np.int64)])
    types = list(dt.TIMESTAMPS)
    blob = np.repeat(ts.astype("<i8"), len(types)).view(np.uint8)
    base = np.arange(n, dtype=np.uint64) * (8 * len(types))
    lens = np.full(n * len(types), 8, np.uint32)
    check_batch(oracle, torch, dev, types, blob, base, lens)


def test_bad_size_sets_status(torch_dev):
    torch, dev = torch_dev
    types = [dt.HYPERDATATYPE_STRING, dt.HYPERDATATYPE_INT64]
    blob = np.zeros(64, np.uint8)
    base = np.array([0, 16], np.uint64)
    lens = np.array([4, 8, 4, 5], np.uint32)  # object 1 attr 1 is 5 bytes
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    got = gpu_hash(torch, dev, types, blob, base, lens, status=status)
    assert int(status.item()) == 1 << _lib.HDX_E_BADSIZE
    assert got[1, 1] == 0
    with pytest.raises(hdx.HdxError) as e:
        hdx.hash_batch_host(types, blob, base, lens)
    assert e.value.status == _lib.HDX_E_BADSIZE
    with pytest.raises(hdx.HdxError) as e:
        hdx.hash(dt.HYPERDATATYPE_FLOAT, b"\0" * 7)
    assert e.value.status == _lib.HDX_E_BADSIZE


@pytest.mark.parametrize("variant", [12, 21, 25, 44, 46, 212, 280, 281, 282, 285, 286])
def test_bad_size_every_variant(oracle, torch_dev, variant):
    """A config-2 batch (key + 4 int64) with one 5-byte int64 in a late
    object: HDX_E_BADSIZE, that coordinate 0, every other coordinate the
    oracle's (the deferred-string forms hash the key in its own pass)."""
    torch, dev = torch_dev
    types, blob, base, lens = synth.make_batch_host("cfg2", 3001, seed=8)
    A = len(types)
    want, _ = oracle.hash_batch(types, blob, base, lens)
    lens = lens.copy()
    victim = 2900 * A + 3
    assert lens[victim] == 8
    lens[victim] = 5
    with _lib.debug_library(variant):
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        got = gpu_hash(torch, dev, types, blob, base, lens, status=status)
    assert int(status.item()) == 1 << _lib.HDX_E_BADSIZE
    got = np.asarray(got).reshape(-1)
    assert got[victim] == 0
    ok = np.ones(len(got), bool)
    ok[victim] = False
    # the shortened value moves the victim object's last attribute (bases are
    # explicit, so no other object moves): compare every other object
    o = victim // A
    ok[o * A:(o + 1) * A] = False
    assert np.array_equal(got[ok], want.reshape(-1)[ok])


def test_bad_type_rejected_before_launch(torch_dev):
    torch, dev = torch_dev
    b, o, L = to_dev(torch, dev, np.zeros(8, np.uint8), np.zeros(1, np.uint64),
                     np.array([8], np.uint32))
    with pytest.raises(hdx.HdxError) as e:
        hdx.hash_batch([dt.HYPERDATATYPE_GENERIC], b, o, L)
    assert e.value.status == _lib.HDX_E_BADTYPE


def test_host_path_matches_device_path(oracle, torch_dev):
    torch, dev = torch_dev
    types, blob, base, lens = synth.make_batch_host("cfg3b", 20000, seed=4)
    want, _ = oracle.hash_batch(types, blob, base, lens)
    assert np.array_equal(hdx.hash_batch_host(types, blob, base, lens), want)


def test_host_path_multichunk(oracle, torch_dev):
    """> 2 pipeline chunks (128 MiB each) through the two-stream host path."""
    torch, dev = torch_dev
    types, blob, base, lens = synth.make_batch_host("cfg3a", 300000, seed=8)  # ~326 MB
    got = hdx.hash_batch_host(types, blob, base, lens)
    idx = np.random.default_rng(0).choice(len(base), 3000, replace=False)
    idx.sort()
    sub_base = base[idx]
    sub_lens = lens.reshape(len(base), -1)[idx].ravel()
    want, _ = oracle.hash_batch(types, blob, sub_base, sub_lens)
    assert np.array_equal(got[idx], want)


def test_host_path_bad_size_in_a_late_chunk(oracle, torch_dev):
    """Validation runs chunk by chunk inside the pipeline: a mis-sized numeric
    in the third chunk fails the call with HDX_E_BADSIZE after the copies in
    flight have landed; the objects of the first chunk are hashed, the last
    objects untouched."""
    torch, dev = torch_dev
    types, blob, base, lens = synth.make_batch_host("cfg2", 3_000_000, seed=9)  # ~290 MB, 3 chunks
    A = len(types)
    lens = lens.copy()
    bad = 2_900_000
    lens[bad * A + 2] = 5  # an INT64 of 5 bytes
    out = np.full((len(base), A), 0x5A5A5A5A5A5A5A5A, np.uint64)
    with pytest.raises(hdx.HdxError) as e:
        hdx.hash_batch_host(types, blob, base, lens, out=out)
    assert e.value.status == _lib.HDX_E_BADSIZE
    want, _ = oracle.hash_batch(types, blob, base[:1000], lens[:1000 * A])
    assert np.array_equal(out[:1000], want.reshape(1000, A))
    assert (out[-1000:] == 0x5A5A5A5A5A5A5A5A).all()


def test_device_generator_matches_host_generator(torch_dev):
    torch, dev = torch_dev
    for cfg in ("cfg2", "cfg3b", "mixed"):
        t1, b1, o1, L1 = synth.make_batch_host(cfg, 2000, seed=21, first=12345)
        t2, b2, o2, L2 = synth.make_batch_device(cfg, 2000, seed=21, first=12345, device=dev)
        assert np.array_equal(t1, t2)
        assert np.array_equal(L1, L2.cpu().numpy().view(np.uint32))
        assert np.array_equal(o1, o2.cpu().numpy().view(np.uint64))
        assert np.array_equal(b1, b2.cpu().numpy())


@pytest.mark.parametrize("cfg", ["cfg3a", "cfg3b"])
def test_full_size_sampled(oracle, torch_dev, cfg):
    """BASELINE size (10M objects, ~10.9 GB in HBM): sampled parity + determinism."""
    torch, dev = torch_dev
    n = 10_000_000
    types, blob, base, lens = synth.make_batch_device(cfg, n, device=dev)
    c1 = hdx.hash_batch(types, blob, base, lens)
    c2 = hdx.hash_batch(types, blob, base, lens)
    torch.cuda.synchronize()
    assert torch.equal(c1, c2)
    A = len(types)
    idx = np.unique(np.concatenate([np.arange(64), n - 1 - np.arange(64),
                                    np.random.default_rng(1).choice(n, 4000, replace=False)]))
    ti = torch.from_numpy(idx).to(dev)
    sb = base[ti].cpu().numpy().view(np.uint64)
    sl = lens.view(n, A)[ti].cpu().numpy().view(np.uint32)
    sizes = sl.astype(np.uint64).sum(axis=1)
    # gather the sampled objects into a compact host blob
    parts, nb, pos = [], np.zeros(len(idx), np.uint64), 0
    for k in range(len(idx)):
        parts.append(blob[int(sb[k]):int(sb[k] + sizes[k])].cpu().numpy())
        nb[k] = pos
        pos += int(sizes[k])
    want, err = oracle.hash_batch(types, np.concatenate(parts), nb, sl.ravel())
    assert err == 0
    got = c1[ti].cpu().numpy().view(np.uint64)
    assert np.array_equal(got, want)
    del blob, base, lens, c1, c2
    torch.cuda.empty_cache()


VARIANTS = [12, 18, 19, 20, 21, 25, 26, 30, 31, 35, 37, 38, 39, 44, 45, 46,
            200, 201, 202, 203, 204, 205, 206, 210, 211, 212, 214, 215, 216, 219, 239, 240, 242, 244, 245, 246, 255, 256,
            257, 258, 259, 270, 273, 274, 275, 276, 278, 279, 280, 281, 282, 283, 284, 285, 286, 300]


@pytest.mark.parametrize("variant", [200, 201, 202, 203, 204, 205, 206, 210, 211, 212, 214, 215, 216, 219, 239, 240, 242, 244, 245, 246, 255,
                                     256, 257, 258, 259, 270, 273, 274, 275, 276, 278, 279, 287, 293, 294, 295, 296, 298])
def test_wave_staged_layouts(oracle, torch_dev, variant):
    """The wave-staged kernel (hdx_wstage.hip) stages a group's span only when
    its objects are back to back and fit the window: gaps after some objects
    (an early DMA that turns out unusable), one oversized object per group,
    and a batch whose last object ends at the blob's last byte all give the
    reference's coordinates."""
    torch, dev = torch_dev
    rng = np.random.default_rng(variant)
    with _lib.debug_library(variant):
        for n in (1, 6, 7, 8, 64, 2001):
            types, blob, base, lens = synth.make_batch_host("cfg3b", n, seed=n)
            check_batch(oracle, torch, dev, types, blob, base, lens)
            # gaps: shift every object after a random cut by a few bytes
            gap = np.cumsum(rng.integers(0, 2, n) * rng.integers(1, 40, n)).astype(np.uint64)
            nb = np.zeros(int(base[-1] + gap[-1]) + int(lens.reshape(n, -1)[-1].sum()) + 1, np.uint8)
            A = len(types)
            sz = lens.reshape(n, A).astype(np.uint64).sum(axis=1)
            for i in range(n):
                nb[int(base[i] + gap[i]):int(base[i] + gap[i] + sz[i])] = blob[int(base[i]):int(base[i] + sz[i])]
            check_batch(oracle, torch, dev, types, nb[:-1], base + gap, lens)
        # objects far larger than any window (keys of 200..4000 bytes + attrs)
        types, blob, base, lens = synth.make_batch_host("keyonly_long", 300, seed=3)
        check_batch(oracle, torch, dev, types, blob, base, lens)
        types, blob, base, lens = synth.make_batch_host("mixed", 700, seed=4)
        check_batch(oracle, torch, dev, types, blob, base, lens)


@pytest.mark.parametrize("variant", [212, 255, 275, 276])
def test_wave_staged_long_strings(oracle, torch_dev, variant):
    """Packed one-string objects, mostly of 0..128 bytes with a few of
    193..1000 per wave (0, 1, a few and many strings past two CityHash loop
    blocks per wave), spans that fit the window and spans that do not, object
    counts that leave waves and workgroups partial."""
    torch, dev = torch_dev
    rng = np.random.default_rng(17)
    with _lib.debug_library(variant):
        for n, p_long in ((63, 0.0), (64, 0.02), (1000, 0.05), (4097, 0.1), (777, 0.5), (300, 1.0)):
            L = rng.integers(0, 129, n).astype(np.uint32)
            longs = rng.random(n) < p_long
            L[longs] = rng.integers(193, 1001, int(longs.sum())).astype(np.uint32)
            lead = int(rng.integers(0, 16))
            base = (lead + np.concatenate([[0], np.cumsum(L[:-1].astype(np.uint64))])).astype(np.uint64)
            blob = rng.integers(0, 256, lead + int(L.sum()), dtype=np.uint8)
            check_batch(oracle, torch, dev, [dt.HYPERDATATYPE_STRING], blob, base, L)


@pytest.mark.parametrize("variant", VARIANTS)
def test_every_kernel_variant_matches_oracle(oracle, torch_dev, variant):
    """The automatic policy picks among these per schema and size (DESIGN.md
    §4.3), and scripts/ab_variants.py times them: each must be bit-exact on
    every config, on ragged object counts and on shuffled objects."""
    torch, dev = torch_dev
    with _lib.debug_library(variant):
        for cfg, n in [("cfg1", 777), ("cfg2", 1001), ("cfg3a", 257), ("cfg3b", 1500),
                       ("mixed", 900), ("wide", 131), ("keyonly_long", 70)]:
            types, blob, base, lens = synth.make_batch_host(cfg, n, seed=variant * 100 + n)
            check_batch(oracle, torch, dev, types, blob, base, lens)
        # every string length 0..200 (all regimes, 1..3 loop blocks) at every
        # byte alignment, the last value ending at the blob's last byte
        rng = np.random.default_rng(variant)
        L = np.repeat(np.arange(201, dtype=np.uint32), 16)
        base = np.arange(len(L), dtype=np.uint64) * 224 + np.tile(np.arange(16, dtype=np.uint64), 201)
        blob = rng.integers(0, 256, int(base[-1]) + 200, dtype=np.uint8)
        check_batch(oracle, torch, dev, [dt.HYPERDATATYPE_STRING], blob, base, L)
        types, blob, base, lens = synth.make_batch_host("cfg3b", 999, seed=5)
        perm = np.random.default_rng(variant).permutation(999)
        A = len(types)
        check_batch(oracle, torch, dev, types, blob, base[perm],
                    lens.reshape(999, A)[perm].reshape(-1))
