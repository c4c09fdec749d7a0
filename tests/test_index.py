"""Secondary-index keys and search pruning.

Oracle (CPU): index keys pinned to the reference's known answers
(tests/golden/reference_values.json) and to oracle/_ref's
ordered encoding when built; byte order of keys == value order; the
lookup_search region loop on hand-built tables.  The search loop itself has no
reference test: parity unpinned beyond the hashes it consumes.
GPU: hdx_index_encode_device and hdx_search_regions against the oracle."""
import json
import os
import struct

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "reference_values.json")
INT64, FLOAT, STRING = 9218, 9219, 9217
TIMESTAMPS = list(range(9473, 9479))


def _le(kind, value):
    if kind == "empty":
        return b""
    if kind == "int64":
        return struct.pack("<q", value)
    if kind == "float":  # bit pattern of the double, hex
        return struct.pack("<Q", int(value, 16))
    return None


def test_oracle_index_keys_pinned_to_reference_values(oracle):
    """INT64 keys are be64(hash(INT64, v)) and FLOAT keys be64(hash(FLOAT, v))
    ++ le(v): check every numeric reference value of SURVEY §8c."""
    cases = json.load(open(GOLDEN))["scalars"]
    seen = 0
    for c in cases:
        if c["type"] not in (INT64, FLOAT):
            continue
        v = _le(c["kind"], c["value"])
        if v is None:
            continue
        key, err = oracle.index_encode(c["type"], v)
        assert err == 0
        assert key[:8] == bytes.fromhex(c["hash"])
        if c["type"] == FLOAT:
            assert key[8:] == (v if len(v) == 8 else bytes(8))
        seen += 1
    assert seen >= 8


def test_oracle_timestamp_keys_are_int64_keys(oracle):
    """index_encoding_timestamp delegates to the int64 encoding
    (daemon/index_timestamp.cc:79-82), not the calendar hash."""
    for t in TIMESTAMPS:
        for v in (b"", struct.pack("<q", 1420666849000000), struct.pack("<q", -1)):
            assert oracle.index_encode(t, v) == oracle.index_encode(INT64, v)


def test_oracle_index_keys_match_reference_build(oracle):
    ref = oracle.ref_lib()
    if ref is None:
        pytest.skip("oracle/_ref not built (reference sources absent)")
    rng = np.random.default_rng(5)
    for x in rng.integers(-2**63, 2**63, 2000, dtype=np.int64):
        key, _ = oracle.index_encode(INT64, struct.pack("<q", int(x)))
        assert key == struct.pack(">Q", ref.ref_ordered_encode_int64(int(x)))
    for x in rng.standard_normal(2000) * 10.0 ** rng.integers(-300, 300, 2000):
        key, _ = oracle.index_encode(FLOAT, struct.pack("<d", x))
        assert key[:8] == struct.pack(">Q", ref.ref_ordered_encode_double(float(x)))


def test_oracle_index_key_byte_order_is_value_order(oracle):
    """The reason the index keys are hashes: memcmp order == numeric order."""
    rng = np.random.default_rng(9)
    ints = np.sort(np.concatenate([rng.integers(-2**63, 2**63, 3000, dtype=np.int64),
                                   np.array([-2**63, -1, 0, 1, 2**63 - 1], np.int64)]))
    keys = [oracle.index_encode(INT64, struct.pack("<q", int(x)))[0] for x in ints]
    assert keys == sorted(keys)
    fl = np.concatenate([rng.standard_normal(3000) * 10.0 ** rng.integers(-300, 300, 3000),
                         [-np.inf, np.inf, 0.0, 5e-324, -5e-324, 1.0, -1.0]])
    fl = np.sort(fl)
    keys = [oracle.index_encode(FLOAT, struct.pack("<d", float(x)))[0][:8] for x in fl]
    assert keys == sorted(keys)


def test_oracle_index_rejects_bad_sizes_and_types(oracle):
    assert oracle.index_encode(INT64, b"abc") == (bytes(8), 2)
    assert oracle.index_encode(FLOAT, b"123456789") == (bytes(16), 2)
    assert oracle.index_encode(STRING, b"abc") == (b"", 0)


# ---- lookup_search region loop -------------------------------------------

def _h(oracle, t, v):
    h, err = oracle.hash_value(t, v)
    assert err == 0
    return h


def test_oracle_search_semantics(oracle):
    """configuration.cc:736-858 on a 1-D INT64 subspace split in 4 and a
    STRING dimension."""
    q = 2**62
    attrs = [3]
    lower = np.array([[0], [q], [2 * q], [3 * q]], np.uint64)
    upper = np.array([[q - 1], [2 * q - 1], [3 * q - 1], [2**64 - 1]], np.uint64)
    i64 = lambda x: struct.pack("<q", x)  # noqa: E731
    # hash(INT64, 0) = 2^63 -> region 2; [0, +inf) keeps regions 2, 3
    inc, cl = oracle.search_regions(attrs, lower, upper, [(3, INT64, i64(0), None)])
    assert list(inc) == [0, 0, 1, 1] and not cl
    # (-inf, -1] keeps 0, 1
    inc, cl = oracle.search_regions(attrs, lower, upper, [(3, INT64, None, i64(-1))])
    assert list(inc) == [1, 1, 0, 0]
    # a range on another attribute prunes nothing
    inc, cl = oracle.search_regions(attrs, lower, upper, [(1, INT64, i64(0), i64(0))])
    assert list(inc) == [1, 1, 1, 1]
    # timestamps are hashed by calendar, not order: never pruned
    inc, cl = oracle.search_regions(attrs, lower, upper, [(3, 9473, i64(5), i64(5))])
    assert list(inc) == [1, 1, 1, 1]
    # invalid range -> empty server list
    inc, cl = oracle.search_regions(attrs, lower, upper, [(3, INT64, i64(0), None, True)])
    assert cl and not inc.any()
    # a STRING point query keeps exactly the region holding its hash
    h = _h(oracle, STRING, b"hyperdex")
    inc, cl = oracle.search_regions(attrs, lower, upper, [(3, STRING, b"hyperdex", b"hyperdex")])
    assert list(inc) == [int(lo <= h <= up) for lo, up in zip(lower[:, 0], upper[:, 0])]
    # a STRING range that is not a point prunes nothing
    inc, _ = oracle.search_regions(attrs, lower, upper, [(3, STRING, b"a", b"b")])
    assert inc.all()
    # an inverted box on a ranged dimension clears the list
    bad_lo = lower.copy()
    bad_lo[2, 0] = upper[2, 0] + np.uint64(1)
    inc, cl = oracle.search_regions(attrs, bad_lo, upper, [(3, INT64, i64(0), None)])
    assert cl


def test_oracle_search_skips_replicaless_regions_first(oracle):
    """configuration.cc:782-785 skips a region without replicas before the
    lower > upper clear of :808-813: an empty box on a replica-less region
    does not clear the search, and the region is never included."""
    q = 2**62
    attrs = [3]
    lower = np.array([[0], [q], [2 * q], [3 * q]], np.uint64)
    upper = np.array([[q - 1], [2 * q - 1], [3 * q - 1], [2**64 - 1]], np.uint64)
    i64 = lambda x: struct.pack("<q", x)  # noqa: E731
    bad_lo = lower.copy()
    bad_lo[1, 0] = upper[1, 0] + np.uint64(1)  # region 1: lower > upper
    rg = [(3, INT64, i64(-2**62), None)]
    inc, cl = oracle.search_regions(attrs, bad_lo, upper, rg)
    assert cl and not inc.any()  # with replicas everywhere the list is cleared
    inc, cl = oracle.search_regions(attrs, bad_lo, upper, rg, has_replicas=[1, 0, 1, 1])
    assert not cl and list(inc) == [0, 0, 1, 1]
    inc, cl = oracle.search_regions(attrs, lower, upper, [], has_replicas=[1, 0, 0, 1])
    assert not cl and list(inc) == [1, 0, 0, 1]
    # an invalid range clears before any region is visited (:762-769)
    inc, cl = oracle.search_regions(attrs, lower, upper, [(3, INT64, i64(0), None, True)], has_replicas=[0] * 4)
    assert cl


def _random_search_case(rng, oracle):
    D = int(rng.integers(1, 5))
    A = 8
    attrs = list(rng.choice(A, size=D, replace=False))
    lo, up = oracle.partition(D, int(rng.choice([4, 8, 64])))
    types = [STRING, INT64, FLOAT, INT64, FLOAT, STRING, 9474, INT64]
    ranges = []
    for a in sorted(rng.choice(A, size=int(rng.integers(0, 5)), replace=False)):
        t = types[a]
        if t == STRING:
            s = bytes(rng.integers(0, 256, int(rng.integers(0, 80)), dtype=np.uint8))
            e = s if rng.random() < 0.7 else s + b"x"
            ranges.append((int(a), t, s, e))
        else:
            fmt = "<d" if t == FLOAT else "<q"
            gen = (lambda: float(rng.standard_normal() * 1e6)) if t == FLOAT else \
                (lambda: int(rng.integers(-2**63, 2**63, dtype=np.int64)))
            s = struct.pack(fmt, gen()) if rng.random() < 0.8 else None
            e = struct.pack(fmt, gen()) if rng.random() < 0.8 else None
            if rng.random() < 0.1:
                s = b""
            ranges.append((int(a), t, s, e))
    if rng.random() < 0.05 and ranges:
        r = list(ranges[0]) + [True]
        ranges[0] = tuple(r)
    if rng.random() < 0.05:
        k = int(rng.integers(0, len(lo)))
        lo[k, 0], up[k, 0] = up[k, 0], lo[k, 0]
    return attrs, lo, up, ranges


def test_oracle_search_random_cases_are_consistent(oracle):
    """A region survives iff every ranged dimension's interval test passes."""
    rng = np.random.default_rng(3)
    for _ in range(200):
        attrs, lo, up, ranges = _random_search_case(rng, oracle)
        inc, cl = oracle.search_regions(attrs, lo, up, ranges)
        if cl:
            assert not inc.any()
            continue
        for r in range(len(lo)):
            keep = True
            for (a, t, s, e, *_) in ranges:
                if a not in attrs:
                    continue
                d = attrs.index(a)
                if t == STRING and s is not None and s == e:
                    h = _h(oracle, t, s)
                    keep &= bool(lo[r, d] <= h <= up[r, d])
                elif t in (INT64, FLOAT):
                    if s is not None:
                        keep &= bool(up[r, d] >= _h(oracle, t, s))
                    if e is not None:
                        keep &= bool(lo[r, d] <= _h(oracle, t, e))
            assert inc[r] == keep


# ---- lookup_search's choice over subspaces (configuration.cc:771-868) -----

def _choose(sets):
    """The reference's rule, restated in Python over per-subspace set sizes:
    the first initialises; a later one replaces if non-empty and <=."""
    chosen, best = -1, None
    for i, n in enumerate(sets):
        if chosen < 0 or (n != 0 and n <= best):
            chosen, best = i, n
    return chosen


def _space(oracle, specs):
    """[(attrs, partitions)] -> [(attrs, lower, upper)] from admin/partition.cc."""
    out = []
    for attrs, parts in specs:
        lo, up = oracle.partition(len(attrs), parts)
        out.append((list(attrs), lo.copy(), up.copy()))
    return out


def test_oracle_search_space_choice(oracle):
    i64 = lambda x: struct.pack("<q", x)  # noqa: E731
    sp = _space(oracle, [([0], 8), ([1], 4), ([2], 4), ([1, 2], 16)])
    # no range names anything: every subspace keeps all its regions; the
    # smallest non-empty set wins and the last of equal sizes wins the tie
    c, inc, cl = oracle.search_space(sp, [])
    assert (c, int(inc.sum()), cl) == (2, 4, False)
    # a range on attr 1 narrows subspace 1 (and 3): [2^62..] keeps 2 of 4 regions
    c, inc, cl = oracle.search_space(sp, [(1, INT64, i64(0), None)])
    assert c == 1 and list(inc) == [0, 0, 1, 1]
    # an empty FIRST subspace is never replaced (initialised, later sets are not <= 0)
    rep = [np.zeros(8, np.uint8), None, None, None]
    c, inc, cl = oracle.search_space(sp, [], has_replicas=rep)
    assert c == 0 and not inc.any() and not cl
    # an empty LATER subspace is never chosen
    rep = [None, np.zeros(4, np.uint8), None, None]
    c, inc, cl = oracle.search_space(sp, [], has_replicas=rep)
    assert c == 2 and inc.sum() == 4
    # no subspaces at all: nothing chosen, not cleared
    assert oracle.search_space([], []) [0] == -1
    # an ill-formed box reached in a LATER subspace clears the whole search
    sp[3][1][5, 1], sp[3][2][5, 1] = sp[3][2][5, 1], sp[3][1][5, 1]
    c, inc, cl = oracle.search_space(sp, [(2, INT64, i64(-5), None)])
    assert c == -1 and cl
    # an invalid range clears before any subspace (:761-768) — with no subspaces too
    c, inc, cl = oracle.search_space(sp[:3], [(0, INT64, i64(0), None, True)])
    assert c == -1 and cl
    c, inc, cl = oracle.search_space([], [(0, INT64, i64(0), None, True)])
    assert c == -1 and cl


def test_search_space_invalid_range_without_subspaces():
    """hdx_search_space rejects an invalid range before looking at any
    subspace (configuration.cc:761-768), so ntables == 0 reports cleared
    (ADVICE r3); no device is touched."""
    import ctypes

    import hyperdex_amd as hdx
    from hyperdex_amd.index import _ranges
    arr = _ranges([(0, INT64, struct.pack("<q", 0), None, True)])
    chosen, servers, cleared = ctypes.c_int32(7), ctypes.c_uint32(7), ctypes.c_int(0)
    assert hdx.lib().hdx_search_space(None, 0, arr, 1, None, ctypes.byref(chosen), None, ctypes.byref(servers),
                                      ctypes.byref(cleared)) == 0
    assert (chosen.value, servers.value, cleared.value) == (-1, 0, 1)


def _random_space(rng, oracle):
    T = int(rng.integers(1, 5))
    specs = [(sorted(rng.choice(8, size=int(rng.integers(1, 4)), replace=False).tolist()),
              int(rng.choice([2, 4, 8, 64]))) for _ in range(T)]
    sp = _space(oracle, specs)
    _, _, _, ranges = _random_search_case(rng, oracle)
    reps = None
    if rng.random() < 0.4:
        reps = [(rng.random(len(lo)) < rng.choice([0.0, 0.5, 1.0])).astype(np.uint8) if rng.random() < 0.7
                else None for _, lo, _ in sp]
    if rng.random() < 0.05:
        k = int(rng.integers(0, T))
        sp[k][1][0, 0], sp[k][2][0, 0] = sp[k][2][0, 0], sp[k][1][0, 0]
    return sp, ranges, reps


def test_oracle_search_space_random_matches_rule(oracle):
    rng = np.random.default_rng(21)
    for _ in range(300):
        sp, ranges, reps = _random_space(rng, oracle)
        c, inc, cl = oracle.search_space(sp, ranges, has_replicas=reps)
        per = [oracle.search_regions(a, lo, up, ranges, has_replicas=None if reps is None else reps[i])
               for i, (a, lo, up) in enumerate(sp)]
        if any(x[1] for x in per):
            assert cl and c == -1
            continue
        assert not cl and c == _choose([int(x[0].sum()) for x in per])
        assert np.array_equal(inc, per[c][0])


@pytest.mark.gpu
def test_gpu_search_space_matches_oracle(oracle):
    import hyperdex_amd as hdx
    rng = np.random.default_rng(23)
    for case in range(150):
        sp, ranges, reps = _random_space(rng, oracle)
        want = oracle.search_space(sp, ranges, has_replicas=reps)
        tables = [hdx.RegionTable(a, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64)) for a, lo, up in sp]
        got = hdx.search_space(tables, ranges, has_replicas=reps)
        for t in tables:
            t.close()
        assert got[0] == want[0] and got[2] == want[2], case
        assert np.array_equal(got[1], want[1]), case
    c, inc, cl = hdx.search_space([], [])
    assert c == -1 and inc.size == 0 and not cl


# ---- GPU -----------------------------------------------------------------

def _column(rng, t, n):
    """n values of type t packed at odd offsets: mostly 8 B, some empty, plus
    the special values the ordered encodings treat specially."""
    vals = []
    for i in range(n):
        r = rng.random()
        if r < 0.05:
            vals.append(b"")
        elif t == FLOAT:
            x = float(rng.standard_normal() * 10.0 ** rng.integers(-300, 300))
            if r < 0.12:
                x = [0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324][i % 7]
            vals.append(struct.pack("<d", x))
        else:
            vals.append(struct.pack("<q", int(rng.integers(-2**63, 2**63, dtype=np.int64))))
    off = np.zeros(n, np.uint64)
    blob = bytearray()
    for i, v in enumerate(vals):
        blob += bytes(int(rng.integers(0, 3)))  # gaps: every alignment
        off[i] = len(blob)
        blob += v
    return vals, np.frombuffer(bytes(blob) + bytes(16), np.uint8), off, \
        np.array([len(v) for v in vals], np.uint32)


@pytest.mark.gpu
@pytest.mark.parametrize("t", [INT64, FLOAT, 9473, 9478])
@pytest.mark.parametrize("n", [1, 255, 257, 20000])
def test_gpu_index_encode_matches_oracle(oracle, t, n):
    import torch

    import hyperdex_amd as hdx
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(n + t)
    vals, blob, off, lens = _column(rng, t, n)
    want = b"".join(oracle.index_encode(t, v)[0] for v in vals)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    got = hdx.index_encode(t, torch.from_numpy(blob.copy()).to(dev),
                           torch.from_numpy(off.view(np.int64)).to(dev),
                           torch.from_numpy(lens.view(np.int32)).to(dev), status=status)
    torch.cuda.synchronize()
    assert got.shape == (n, hdx.index_key_size(t))
    assert got.cpu().numpy().tobytes() == want
    assert int(status.item()) == 0


@pytest.mark.gpu
def test_gpu_index_encode_bad_sizes_and_types():
    import torch

    import hyperdex_amd as hdx
    dev = torch.device("cuda", 0)
    blob = torch.arange(64, dtype=torch.uint8, device=dev)
    off = torch.tensor([0, 8, 20], dtype=torch.int64, device=dev)
    lens = torch.tensor([8, 3, 8], dtype=torch.int32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    got = hdx.index_encode(INT64, blob, off, lens, status=status).cpu().numpy()
    assert int(status.item()) & (1 << 2)
    assert not got[1].any() and got[0].any() and got[2].any()
    assert hdx.index_key_size(STRING) == 0 and hdx.index_key_size(FLOAT) == 16
    with pytest.raises(hdx.HdxError):
        hdx.index_encode(STRING, blob, off, lens)
    with pytest.raises(hdx.HdxError):
        hdx.index_encode(12345, blob, off, lens)


@pytest.mark.gpu
def test_gpu_search_regions_matches_oracle(oracle):
    import hyperdex_amd as hdx
    rng = np.random.default_rng(11)
    for case in range(300):
        attrs, lo, up, ranges = _random_search_case(rng, oracle)
        rep = None
        if case % 3 == 1:  # some regions without replicas (incl. empty boxes)
            rep = (rng.random(len(lo)) < 0.7).astype(np.uint8)
        want, wcl = oracle.search_regions(attrs, lo, up, ranges, has_replicas=rep)
        table = hdx.RegionTable(attrs, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64))
        got, cl = hdx.search_regions(table, ranges, has_replicas=rep)
        table.close()
        assert cl == wcl, case
        assert np.array_equal(got, want), case


@pytest.mark.gpu
def test_gpu_search_replicaless_empty_box(oracle):
    """A replica-less region with an empty box (lower > upper) on a ranged
    dimension neither clears the search nor appears in it."""
    import hyperdex_amd as hdx
    lo, up = oracle.partition(2, 16)
    lo, up = lo.copy(), up.copy()
    lo[5, 1], up[5, 1] = up[5, 1], lo[5, 1]
    rep = np.ones(len(lo), np.uint8)
    rg = [(4, INT64, struct.pack("<q", -5), struct.pack("<q", 2**50))]
    table = hdx.RegionTable([2, 4], lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64))
    inc, cl = hdx.search_regions(table, rg, has_replicas=rep)
    assert cl and not inc.any()
    rep[5] = 0
    inc, cl = hdx.search_regions(table, rg, has_replicas=rep)
    want, wcl = oracle.search_regions([2, 4], lo, up, rg, has_replicas=rep)
    assert not cl and not wcl and inc[5] == 0 and np.array_equal(inc, want) and inc.any()
    table.close()


@pytest.mark.gpu
def test_gpu_search_regions_point_queries(oracle):
    """Every STRING point query on a 64-region key subspace keeps exactly one
    region: the one lookup_region would route the key to."""
    import hyperdex_amd as hdx
    lo, up = oracle.partition(1, 64)
    ids = np.arange(1, 65, dtype=np.uint64)
    table = hdx.RegionTable([0], lo, up, ids)
    rng = np.random.default_rng(1)
    for _ in range(50):
        key = bytes(rng.integers(0, 256, int(rng.integers(0, 100)), dtype=np.uint8))
        inc, cl = hdx.search_regions(table, [(0, STRING, key, key)])
        assert not cl and inc.sum() == 1
        coords = np.array([[_h(oracle, STRING, key)]], np.uint64)
        assert ids[np.argmax(inc)] == oracle.lookup_region([0], lo, up, ids, coords)[0]
    # pruning follows the range's type, not the dimension's
    rg = [(0, INT64, struct.pack("<q", 1), struct.pack("<q", 2**40))]
    inc, cl = hdx.search_regions(table, rg)
    assert np.array_equal(inc, oracle.search_regions([0], lo, up, rg)[0]) and 0 < inc.sum() < 64
    with pytest.raises(hdx.HdxError):  # a mis-sized numeric endpoint is an error
        hdx.search_regions(table, [(0, INT64, b"123", None)])
    table.close()
