"""Synthetic object batches (SURVEY §8d shapes), on the host (numpy) or in HBM.

The device generator is hyperdex_amd/csrc/hdx_synth.hip; this module restates
the same counter-based rules in numpy so tests can rebuild any batch on the
host.  RNG: splitmix64 finaliser over
    R(stream, k) = mix64(seed + stream * 0xd1b54a32d192ed03 + (k + 1) * 0x9e3779b97f4a7c15)
Streams: 1 uniform lengths, 2(+first<<8) blob bytes, 3 numeric values,
4 numeric special-value selector.  Default seed 0x4859504552444558 ("HYPERDEX").
"""
import ctypes
from dataclasses import dataclass
from typing import List, Tuple

import numpy as np

from . import datatypes as dt

SEED = 0x4859504552444558
GOLD = np.uint64(0x9e3779b97f4a7c15)
SALT = np.uint64(0xd1b54a32d192ed03)

FIXED, UNIFORM, NUMERIC = 0, 1, 2


@dataclass(frozen=True)
class Rule:
    type: int
    kind: int
    lo: int = 0
    hi: int = 0


def _s(L):  # key STRING fixed 64 B
    return Rule(dt.HYPERDATATYPE_STRING, FIXED, L, L)


def _n(t):
    return Rule(t, NUMERIC, 8, 8)


# SURVEY §8d configs (config 4 = 3b sharded; config 5 reuses 3b).
CONFIGS = {
    "cfg1": [_s(64)],
    "cfg2": [_s(64)] + [_n(dt.HYPERDATATYPE_INT64)] * 4,
    "cfg3a": [_s(64)] * 17,
    "cfg3b": ([_s(64)] + [Rule(dt.HYPERDATATYPE_STRING, UNIFORM, 0, 195)] * 10
              + [_n(dt.HYPERDATATYPE_INT64)] * 3 + [_n(dt.HYPERDATATYPE_FLOAT)] * 3),
    # test-only: every hashable type, non-hashable containers, every CityHash regime
    "mixed": ([Rule(dt.HYPERDATATYPE_STRING, UNIFORM, 0, 300)]
              + [Rule(dt.HYPERDATATYPE_STRING, UNIFORM, 0, 20)]
              + [_n(dt.HYPERDATATYPE_INT64), _n(dt.HYPERDATATYPE_FLOAT)]
              + [_n(t) for t in dt.TIMESTAMPS]
              + [Rule(dt.HYPERDATATYPE_LIST_STRING, UNIFORM, 0, 40),
                 Rule(dt.HYPERDATATYPE_DOCUMENT, UNIFORM, 0, 24),
                 Rule(dt.HYPERDATATYPE_MAP_INT64_FLOAT, FIXED, 16, 16),
                 Rule(dt.HYPERDATATYPE_STRING, UNIFORM, 60, 140)]),
    # test-only: many attributes, all strings of every length class
    "wide": [Rule(dt.HYPERDATATYPE_STRING, UNIFORM, 0, 130)] * 70,
    "keyonly_long": [Rule(dt.HYPERDATATYPE_STRING, UNIFORM, 200, 4000)],
    # measurement-only: 17 attributes of one CityHash regime / loop count each
    "u8": [_s(8)] * 17, "u24": [_s(24)] * 17, "u48": [_s(48)] * 17, "u100": [_s(100)] * 17,
    "u150": [_s(150)] * 17, "u190": [_s(190)] * 17,
    "num": [_n(dt.HYPERDATATYPE_INT64)] * 17, "flt": [_n(dt.HYPERDATATYPE_FLOAT)] * 17,
    # measurement-only: config 3b with its strings capped at 2 / 1 CityHash loop trips
    "m3b192": ([_s(64)] + [Rule(dt.HYPERDATATYPE_STRING, UNIFORM, 0, 192)] * 10
               + [_n(dt.HYPERDATATYPE_INT64)] * 3 + [_n(dt.HYPERDATATYPE_FLOAT)] * 3),
    "m3b128": ([_s(64)] + [Rule(dt.HYPERDATATYPE_STRING, UNIFORM, 0, 128)] * 10
               + [_n(dt.HYPERDATATYPE_INT64)] * 3 + [_n(dt.HYPERDATATYPE_FLOAT)] * 3),
    # measurement-only: config 3b's attribute mix repeated to 200 / 1000 attributes
    # (the A > 128 gather kernel 44 and the A > 256 wide kernel)
    "w200": [_s(64)] + ([Rule(dt.HYPERDATATYPE_STRING, UNIFORM, 0, 195)] * 10
                        + [_n(dt.HYPERDATATYPE_INT64)] * 3 + [_n(dt.HYPERDATATYPE_FLOAT)] * 3) * 12
                      + [_s(64)] * 7,
    "w1000": [_s(64)] + ([Rule(dt.HYPERDATATYPE_STRING, UNIFORM, 0, 195)] * 10
                         + [_n(dt.HYPERDATATYPE_INT64)] * 3 + [_n(dt.HYPERDATATYPE_FLOAT)] * 3) * 62
                       + [_s(64)] * 7,
}


def payload_bytes_per_object(name: str) -> float:
    tot = 0.0
    for r in CONFIGS[name]:
        tot += (r.lo + r.hi) / 2 if r.kind == UNIFORM else (8 * 0.99 if r.kind == NUMERIC else r.lo)
    return tot


def mix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return z ^ (z >> np.uint64(31))


def rnd(seed: int, stream: int, k: np.ndarray) -> np.ndarray:
    k = np.asarray(k, dtype=np.uint64)
    with np.errstate(over="ignore"):
        base = np.uint64(seed) + np.uint64(stream & 0xffffffffffffffff) * SALT
        return mix64(base + (k + np.uint64(1)) * GOLD)


def lengths(rules: List[Rule], n: int, seed: int = SEED, first: int = 0) -> np.ndarray:
    A = len(rules)
    f = (np.uint64(first) * np.uint64(A)) + np.arange(n * A, dtype=np.uint64)
    out = np.empty(n * A, dtype=np.uint32)
    j = np.arange(n * A) % A
    for jj, r in enumerate(rules):
        m = j == jj
        if r.kind == FIXED:
            out[m] = r.lo
        elif r.kind == UNIFORM:
            out[m] = (r.lo + rnd(seed, 1, f[m]) % np.uint64(r.hi - r.lo + 1)).astype(np.uint32)
        else:
            out[m] = np.where(rnd(seed, 4, f[m]) % np.uint64(100) == 0, 0, 8).astype(np.uint32)
    return out


def numeric_values(t: int, seed: int, f: np.ndarray) -> np.ndarray:
    """Mirror of synth_numeric() in hdx_synth.hip (uint64 bit patterns)."""
    sel = rnd(seed, 4, f) % np.uint64(100)
    v = rnd(seed, 3, f)
    FRAC, SIGN = np.uint64(0x000fffffffffffff), np.uint64(0x8000000000000000)
    if t == dt.HYPERDATATYPE_INT64:
        mm = np.where(v & np.uint64(1), np.uint64(0x7fffffffffffffff), SIGN)
        return np.where(sel == 1, mm, v)
    if t == dt.HYPERDATATYPE_FLOAT:
        e = np.uint64(963) + ((v >> np.uint64(52)) & np.uint64(0x7f)) % np.uint64(121)
        out = (v & SIGN) | (e << np.uint64(52)) | (v & FRAC)
        spec = {1: np.zeros_like(v), 2: np.full_like(v, SIGN),
                3: np.full_like(v, 0x7ff0000000000000), 4: np.full_like(v, 0xfff0000000000000),
                5: np.uint64(0x7ff8000000000000) | (v & np.uint64(0x8007ffffffffffff)),
                6: (v & FRAC) | np.uint64(1), 7: SIGN | (v & FRAC) | np.uint64(1)}
        for s, val in spec.items():
            out = np.where(sel == s, val, out)
        return out
    return np.where(sel < 50, v & np.uint64((1 << 51) - 1), v)


def object_bases(attr_len: np.ndarray, A: int) -> Tuple[np.ndarray, int]:
    sizes = attr_len.reshape(-1, A).astype(np.uint64).sum(axis=1)
    base = np.zeros(len(sizes), dtype=np.uint64)
    if len(sizes) > 1:
        base[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    total = int(sizes.sum()) if len(sizes) else 0
    return base, total


def blob_bytes(seed: int, first: int, nbytes: int) -> np.ndarray:
    words = rnd(seed, 2 + (first << 8), np.arange((nbytes + 7) // 8, dtype=np.uint64))
    return words.view(np.uint8)[:nbytes].copy()


def make_batch_host(name_or_rules, n: int, seed: int = SEED, first: int = 0):
    """(types u32[A], blob u8, obj_base u64[n], attr_len u32[n*A]) on the host,
    byte-identical to make_batch_device(..) of the same arguments."""
    rules = CONFIGS[name_or_rules] if isinstance(name_or_rules, str) else list(name_or_rules)
    A = len(rules)
    L = lengths(rules, n, seed, first)
    base, total = object_bases(L, A)
    blob = blob_bytes(seed, first, total)
    Lm = L.reshape(n, A)
    offs = base[:, None] + np.concatenate(
        [np.zeros((n, 1), np.uint64), np.cumsum(Lm, axis=1, dtype=np.uint64)[:, :-1]], axis=1)
    for j, r in enumerate(rules):
        if r.kind != NUMERIC:
            continue
        rows = np.nonzero(Lm[:, j] == 8)[0]
        f = (np.uint64(first) + rows.astype(np.uint64)) * np.uint64(A) + np.uint64(j)
        vals = numeric_values(r.type, seed, f).astype("<u8").view(np.uint8).reshape(-1, 8)
        idx = offs[rows, j].astype(np.int64)[:, None] + np.arange(8)[None, :]
        blob[idx] = vals
    types = np.array([r.type for r in rules], dtype=np.uint32)
    return types, blob, base, L


def c_rules(rules: List[Rule]):
    from ._lib import SynthRule
    arr = (SynthRule * len(rules))()
    for i, r in enumerate(rules):
        arr[i] = SynthRule(r.type, r.kind, r.lo, r.hi)
    return arr


def make_batch_device(name_or_rules, n: int, seed: int = SEED, first: int = 0, device=None,
                      pad: int = 0):
    """Generate the batch directly in HBM (torch tensors on `device`).

    Returns (types np.u32[A], blob u8, obj_base i64[n], attr_len i32[n*A]);
    obj_base/attr_len are int64/int32 tensors holding the u64/u32 values."""
    import torch

    from ._lib import check, lib

    rules = CONFIGS[name_or_rules] if isinstance(name_or_rules, str) else list(name_or_rules)
    A = len(rules)
    device = device or torch.device("cuda", torch.cuda.current_device())
    if A > 64:  # the device generator's rule table holds 64: the host generator, copied
        types, hb, hbase, hL = make_batch_host(rules, n, seed, first)
        blob = torch.empty(len(hb) + pad, dtype=torch.uint8, device=device)
        blob[:len(hb)] = torch.from_numpy(hb).to(device)
        return (types, blob, torch.from_numpy(hbase.view(np.int64)).to(device),
                torch.from_numpy(hL.view(np.int32)).to(device))
    cr = c_rules(rules)
    stream = torch.cuda.current_stream(device).cuda_stream
    attr_len = torch.empty(n * A, dtype=torch.int32, device=device)
    check(lib().hdx_synth_lengths(cr, A, seed, first, n, attr_len.data_ptr(), stream))
    sizes = attr_len.view(n, A).to(torch.int64).sum(dim=1)
    obj_base = torch.zeros(n, dtype=torch.int64, device=device)
    if n > 1:
        obj_base[1:] = torch.cumsum(sizes[:-1], dim=0)
    total = int(sizes.sum().item()) if n else 0
    blob = torch.empty(total + pad, dtype=torch.uint8, device=device)
    check(lib().hdx_synth_fill(cr, A, seed, first, n, obj_base.data_ptr(), attr_len.data_ptr(),
                               blob.data_ptr(), total, stream))
    types = np.array([r.type for r in rules], dtype=np.uint32)
    return types, blob, obj_base, attr_len


def encode_values_host(types, blob, obj_base, attr_len, first_version=0):
    """daemon/datalayer_encodings.cc:139-166 (encode_value) on the host: the
    packed batch's attribute 0 becomes the key, attributes 1..A-1 the value.
    Returns (keys, key_off, key_len, vals, val_off, val_len) numpy arrays."""
    A = len(types)
    n = len(obj_base)
    Lm = attr_len.reshape(n, A).astype(np.uint64)
    key_off = obj_base.astype(np.uint64)
    key_len = Lm[:, 0].astype(np.uint32)
    val_len = (10 + (4 + Lm[:, 1:]).sum(axis=1)).astype(np.uint32)
    val_off = np.zeros(n, np.uint64)
    if n > 1:
        val_off[1:] = np.cumsum(val_len[:-1].astype(np.uint64))
    vals = np.zeros(int(val_len.astype(np.uint64).sum()) if n else 0, np.uint8)
    for i in range(n):
        o = int(val_off[i])
        vals[o:o + 8] = np.frombuffer(int(first_version + i).to_bytes(8, "big"), np.uint8)
        vals[o + 8:o + 10] = np.frombuffer((A - 1).to_bytes(2, "big"), np.uint8)
        o += 10
        src = int(obj_base[i]) + int(Lm[i, 0])
        for j in range(1, A):
            L = int(Lm[i, j])
            vals[o:o + 4] = np.frombuffer(L.to_bytes(4, "big"), np.uint8)
            vals[o + 4:o + 4 + L] = blob[src:src + L]
            o += 4 + L
            src += L
    return blob, key_off, key_len, vals, val_off, val_len


def encode_store_host(types, blob, obj_base, attr_len, first_version=0, layout="records"):
    """encode_values_host's objects in make_encoded_device's "keycol" or
    "records" layout: returns (keys, key_off, key_len, vals, val_off, val_len)."""
    _, _, key_len, vals, val_off, val_len = encode_values_host(types, blob, obj_base, attr_len, first_version)
    n = len(obj_base)
    kl = key_len.astype(np.uint64)

    def exclusive_cumsum(x):
        out = np.zeros(n, np.uint64)
        if n > 1:
            out[1:] = np.cumsum(x[:-1])
        return out
    if layout == "keycol":
        key_off = exclusive_cumsum(kl)
        keys = np.zeros(int(kl.sum()) if n else 0, np.uint8)
        for i in range(n):
            keys[int(key_off[i]):int(key_off[i] + kl[i])] = blob[int(obj_base[i]):int(obj_base[i] + kl[i])]
        return keys, key_off, key_len, vals, val_off, val_len
    assert layout == "records"
    rec = kl + val_len.astype(np.uint64)
    rec_off = exclusive_cumsum(rec)
    store = np.zeros(int(rec.sum()) if n else 0, np.uint8)
    for i in range(n):
        r, k, v = int(rec_off[i]), int(kl[i]), int(val_len[i])
        store[r:r + k] = blob[int(obj_base[i]):int(obj_base[i]) + k]
        store[r + k:r + k + v] = vals[int(val_off[i]):int(val_off[i]) + v]
    return store, rec_off, key_len, store, rec_off + kl, val_len


def make_encoded_device(name_or_rules, n: int, seed: int = SEED, first: int = 0, device=None,
                        layout: str = "columns"):
    """A packed synthetic batch re-encoded as stored objects in HBM (config 5):
    returns (types, keys, key_off, key_len, vals, val_off, val_len).
      "columns": keys = the batch blob (key_off = obj_base: each key in place
                 inside its packed object), values back to back in a new
                 buffer (round 3's layout);
      "keycol":  keys back to back in a key column (key_off = their prefix
                 offsets, SURVEY §8d's "key, obj_base[n+1]"), values back to
                 back beside it;
      "records": one store of records [key][value] back to back (the
                 adjacency of a LevelDB block's key / value entries); keys
                 and vals are the same tensor.
    The last two free the batch blob."""
    import torch

    from ._lib import check, lib

    assert layout in ("columns", "keycol", "records")
    types, blob, obj_base, attr_len = make_batch_device(name_or_rules, n, seed, first, device)
    A = len(types)
    dev = blob.device
    L = attr_len.view(n, A).to(torch.int64)
    key_len = attr_len.view(n, A)[:, 0].contiguous()
    val_len64 = 10 + (4 + L[:, 1:]).sum(dim=1)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def exclusive_cumsum(x):
        out = torch.zeros(n, dtype=torch.int64, device=dev)
        if n > 1:
            out[1:] = torch.cumsum(x[:-1], dim=0)
        return out

    if layout == "columns":
        val_off = exclusive_cumsum(val_len64)
        vals = torch.empty(max(int(val_len64.sum().item()) if n else 0, 1), dtype=torch.uint8, device=dev)
        check(lib().hdx_synth_encode_values(blob.data_ptr(), obj_base.data_ptr(), attr_len.data_ptr(), A, n,
                                            first, val_off.data_ptr(), vals.data_ptr(), stream))
        return (types, blob, obj_base, key_len, vals, val_off, val_len64.to(torch.int32))
    if layout == "records":
        rec_off = exclusive_cumsum(val_len64 + L[:, 0])
        val_off = rec_off + L[:, 0]
        total = int((val_len64 + L[:, 0]).sum().item()) if n else 0
        vals = keys = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
        key_off = rec_off
    else:
        key_off = exclusive_cumsum(L[:, 0])
        val_off = exclusive_cumsum(val_len64)
        keys = torch.empty(max(int(L[:, 0].sum().item()) if n else 0, 1), dtype=torch.uint8, device=dev)
        vals = torch.empty(max(int(val_len64.sum().item()) if n else 0, 1), dtype=torch.uint8, device=dev)
    del L
    check(lib().hdx_synth_encode_store(blob.data_ptr(), obj_base.data_ptr(), attr_len.data_ptr(), A, n, first,
                                       val_off.data_ptr(), vals.data_ptr(), key_off.data_ptr(), keys.data_ptr(),
                                       stream))
    torch.cuda.current_stream(dev).synchronize()
    del blob, obj_base, attr_len
    return (types, keys, key_off, key_len, vals, val_off, val_len64.to(torch.int32))
