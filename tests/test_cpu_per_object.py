"""The per-object entry points of libhdxhash.so (hdx_hash_value / hdx_hash_key /
hdx_hash_object, the C form of common/hash.h:43-55) run on the host CPU
(hyperdex_amd/csrc/hdx_cpu.cpp) and need no GPU.  Pinned to the reference's
own known answers and checked against the oracle on random values:

  * CityHash64: all 300 vectors of cityhash/test/city.cc:63-1265, plus every
    length 0..520 at every alignment 0..15 against the oracle
  * the reference-produced scalars and the whole object of SURVEY.md §8c
  * ordered int64 / double encodings and the timestamp hash on random and
    special bit patterns against the oracle
  * the reference's assert paths (unknown type, mis-sized numerics) -> errors
"""
import json
import os
import struct

import numpy as np
import pytest

import hyperdex_amd as hdx
from hyperdex_amd import _lib, datatypes as dt
from kat_data import kat_data

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def encode_value(kind, value):
    if kind == "empty":
        return b""
    if kind == "bytes":
        return value.encode()
    if kind == "int64":
        return struct.pack("<q", value)
    return struct.pack("<Q", int(value, 16))


def test_cityhash_kat_on_cpu():
    data = kat_data()
    for c in load("cityhash64_kat.json")["cases"]:
        got = hdx.hash(dt.HYPERDATATYPE_STRING, data[c["offset"]:c["offset"] + c["len"]])
        assert got == int(c["cityhash64"], 16), c


def test_every_length_and_alignment_vs_oracle(oracle):
    buf = np.random.default_rng(7).integers(0, 256, 600, dtype=np.uint8).tobytes()
    for n in range(0, 521):
        for a in range(0, 16, 5 if n > 80 else 1):
            s = buf[a:a + n]
            assert hdx.hash(dt.HYPERDATATYPE_STRING, s) == oracle.cityhash64(s), (n, a)


def test_reference_scalars_on_cpu():
    for s in load("reference_values.json")["scalars"]:
        assert hdx.hash(s["type"], encode_value(s["kind"], s["value"])) == int(s["hash"], 16), s


def test_reference_object_on_cpu():
    for o in load("reference_values.json")["objects"]:
        vals = [encode_value(v["kind"], v["value"]) for v in o["values"]]
        got = hdx.hash_object(o["types"], o["key"].encode(), vals)
        assert ["%016x" % c for c in got] == o["hashes"]
        assert hdx.hash_key(o["types"], o["key"].encode()) == int(o["hashes"][0], 16)


SPECIAL_BITS = [0, 1 << 63, 0x7ff0000000000000, 0xfff0000000000000, 0x7ff8000000000000, 0xfff8000000000001,
                0x7ff0000000000001, 1, 0x8000000000000001, 0x000fffffffffffff, 0x800fffffffffffff,
                0x7fefffffffffffff, 0xffefffffffffffff, 0x3ff0000000000000, 0xbff0000000000000,
                0x7fffffffffffffff, 0xffffffffffffffff]


@pytest.mark.parametrize("t", [dt.HYPERDATATYPE_INT64, dt.HYPERDATATYPE_FLOAT] + list(range(9473, 9479)))
def test_numeric_types_vs_oracle(oracle, t):
    rng = np.random.default_rng(t)
    bits = list(rng.integers(0, 2**63, 3000, dtype=np.uint64) * 2 + rng.integers(0, 2, 3000, dtype=np.uint64))
    bits += SPECIAL_BITS
    if t >= 9473:  # timestamps: realistic microsecond values, negatives, >= 2^53
        bits += [1420666849000000, 1389130849000000, (1 << 64) - 1, 9007199254740993, (1 << 53) + 1]
    for b in bits:
        v = struct.pack("<Q", int(b))
        want, err = oracle.hash_value(t, v)
        assert err == 0
        assert hdx.hash(t, v) == want, (t, hex(int(b)))
    want, _ = oracle.hash_value(t, b"")
    assert hdx.hash(t, b"") == want


def test_random_objects_vs_oracle(oracle):
    from hyperdex_amd import synth
    for cfg in ("cfg3b", "mixed", "cfg2"):
        types, blob, base, lens = synth.make_batch_host(cfg, 300)
        A = len(types)
        want, err = oracle.hash_batch(types, blob, base, lens)
        assert err == 0
        for i in range(300):
            L = lens[i * A:(i + 1) * A]
            offs = int(base[i]) + np.concatenate([[0], np.cumsum(L[:-1], dtype=np.int64)])
            parts = [blob[o:o + n].tobytes() for o, n in zip(offs, L)]
            assert hdx.hash_object(types, parts[0], parts[1:]) == list(want[i]), (cfg, i)


def test_reference_assert_paths_return_errors():
    """hash.cc:38 asserts on an unknown type; datatype_int64.cc:233 /
    datatype_float.cc:204 / datatype_timestamp.cc:46 on a value not 0 or 8
    bytes: the C-ABI returns HDX_E_BADTYPE / HDX_E_BADSIZE instead."""
    with pytest.raises(hdx.HdxError) as e:
        hdx.hash(dt.HYPERDATATYPE_GENERIC, b"x")
    assert e.value.status == _lib.HDX_E_BADTYPE
    for t in (dt.HYPERDATATYPE_INT64, dt.HYPERDATATYPE_FLOAT, dt.HYPERDATATYPE_TIMESTAMP_DAY):
        with pytest.raises(hdx.HdxError) as e:
            hdx.hash(t, b"1234")
        assert e.value.status == _lib.HDX_E_BADSIZE
    with pytest.raises(hdx.HdxError) as e:
        hdx.hash_object([dt.HYPERDATATYPE_STRING, dt.HYPERDATATYPE_INT64], b"k", [b"123"])
    assert e.value.status == _lib.HDX_E_BADSIZE
    assert hdx.hash(dt.HYPERDATATYPE_MAP_STRING_INT64, b"\x01\x02\x03") == 0  # not hashable -> 0


def test_cpubench_harness_matches_oracle():
    """bench.py's cpu_per_object leg (tools/libhdxcpubench.so: one
    hdx_hash_object / hdx_hash_key call per object, N threads) computes the
    reference's coordinates; bench.py checks the same against the GPU's."""
    import bench
    from hyperdex_amd import synth
    from oracle import oracle
    for cfg, n in (("cfg1", 5000), ("cfg3b", 3000), ("mixed", 2000)):
        types, blob, base, lens = synth.make_batch_host(cfg, n, seed=11)
        want, err = oracle.hash_batch(types, blob, base, lens)
        assert err == 0
        res = bench.cpu_per_object(types, blob, base, lens, want, 0.05, cfg)
        assert res["verified_vs_gpu"] and res["objects"] == n and res["ns_per_object_1thread"] > 0
