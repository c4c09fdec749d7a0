"""Pins the CPU oracle (oracle/hdx_oracle.c) to the reference's own known answers.

  * CityHash64: all 300 column-0 vectors of cityhash/test/city.cc:63-1265
  * ordered encodings: common/test/ordered_encoding.cc:42-69 exact cases, its
    monotonicity property (:71-122), and — when oracle/_ref is built — the
    reference's ordered_encoding.cc itself on random and special inputs
  * timestamp / whole-object hash: reference-produced values of SURVEY.md §8c
"""
import json
import math
import os
import struct

import numpy as np
import pytest

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


def test_cityhash_kat(oracle):
    data = kat_data()
    kat = load("cityhash64_kat.json")["cases"]
    assert len(kat) == 300
    for c in kat:
        got = oracle.cityhash64(data[c["offset"]:c["offset"] + c["len"]])
        assert got == int(c["cityhash64"], 16), c


def test_reference_scalars(oracle):
    for s in load("reference_values.json")["scalars"]:
        h, err = oracle.hash_value(s["type"], encode_value(s["kind"], s["value"]))
        assert err == 0
        assert h == int(s["hash"], 16), s


def test_reference_object(oracle):
    for o in load("reference_values.json")["objects"]:
        vals = [o["key"].encode()] + [encode_value(v["kind"], v["value"]) for v in o["values"]]
        lens = np.array([len(v) for v in vals], np.uint32)
        blob = np.frombuffer(b"".join(vals), np.uint8)
        coords, err = oracle.hash_batch(o["types"], blob, np.zeros(1, np.uint64), lens)
        assert err == 0
        assert ["%016x" % c for c in coords[0]] == o["hashes"]


def test_ordered_encoding_kat(oracle):
    kat = load("reference_values.json")["ordered_encoding_kat"]
    L = oracle.lib()
    for x, want in kat["int64"]:
        assert L.hdxo_encode_int64(int(x)) == int(want, 16)
    for bits, want in kat["double"]:
        d = struct.unpack("<d", struct.pack("<Q", int(bits, 16)))[0]
        assert L.hdxo_encode_double(d) == int(want, 16)


def test_ordered_double_monotone(oracle):
    """common/test/ordered_encoding.cc:71-122 property on 200k samples."""
    L = oracle.lib()
    rng = np.random.default_rng(48)
    xs = rng.standard_normal(200000) * np.exp(rng.uniform(-700, 700, 200000))
    xs = np.concatenate([xs, [0.0, -0.0, 5e-324, -5e-324, 1.7976931348623157e308,
                              -1.7976931348623157e308]])
    xs = np.sort(xs[np.isfinite(xs)])
    enc = np.array([L.hdxo_encode_double(float(x)) for x in xs], dtype=np.uint64)
    same = xs[1:] == xs[:-1]
    assert np.all((enc[1:] > enc[:-1]) | same)
    assert np.all((enc[1:] == enc[:-1]) == same)
    neg, pos = xs < 0, xs > 0
    assert np.all(enc[neg] < 0x8000000000000001)
    assert np.all(enc[pos] > 0x8000000000000001)


def test_timestamp_granularities_differ(oracle):
    L = oracle.lib()
    t = 1420666849000000
    hs = {L.hdxo_hash_timestamp(g, t) for g in range(9473, 9479)}
    assert len(hs) == 6


def test_bad_sizes_and_types(oracle):
    assert oracle.hash_value(9218, b"1234")[1] == 2
    assert oracle.hash_value(9219, b"123456789")[1] == 2
    assert oracle.hash_value(9473, b"1")[1] == 2
    assert oracle.hash_value(9216, b"")[1] == 1
    assert oracle.hash_value(9416, b"")[1] == 1  # MAP_STRING_KEYONLY: lookup() == NULL
    assert oracle.hash_value(9664, b"secret") == (0, 0)  # macaroon: not hashable


def _ref_or_skip(oracle):
    R = oracle.ref_lib()
    if R is None:
        pytest.skip("oracle/_ref not built (needs /root/reference at build time)")
    return R


def test_against_reference_ordered_encoding(oracle):
    """oracle vs the reference's ordered_encoding.cc compiled unmodified."""
    R = _ref_or_skip(oracle)
    L = oracle.lib()
    rng = np.random.default_rng(7)
    bits = rng.integers(0, 2**64, 50000, dtype=np.uint64)
    specials = [0, 1 << 63, 0x7ff0000000000000, 0xfff0000000000000, 0x7ff8000000000000,
                0xfff8000000000001, 0x7ff0000000000001, 1, (1 << 63) | 1, 0x000fffffffffffff,
                0x800fffffffffffff, 0x0010000000000000, 0x7fefffffffffffff, 0xffefffffffffffff]
    for b in list(bits) + specials:
        b = int(b)
        d = struct.unpack("<d", struct.pack("<Q", b))[0]
        assert L.hdxo_encode_double(d) == R.ref_ordered_encode_double(d), hex(b)
        i = struct.unpack("<q", struct.pack("<Q", b))[0]
        assert L.hdxo_encode_int64(i) == R.ref_ordered_encode_int64(i)


def test_reference_ordered_encoding_selftest():
    """The reference's own test binary, built from its sources, passes."""
    import subprocess
    exe = os.path.join(os.path.dirname(GOLD), "..", "oracle", "_ref", "ordered_encoding_test")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref not built")
    assert subprocess.run([exe], capture_output=True).returncode == 0
