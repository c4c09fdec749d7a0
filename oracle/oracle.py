"""ctypes view of oracle/liboracle.so (TEST INFRASTRUCTURE ONLY).

The CPU restatement of the reference hashing path (oracle/hdx_oracle.c).
Used as the parity checker and as bench.py's cpu_baseline ("port").
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        u64, u32, i64, sz = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int64, ctypes.c_size_t
        vp = ctypes.c_void_p
        L.hdxo_cityhash64.argtypes = [vp, sz]
        L.hdxo_cityhash64.restype = u64
        L.hdxo_encode_int64.argtypes = [i64]
        L.hdxo_encode_int64.restype = u64
        L.hdxo_encode_double.argtypes = [ctypes.c_double]
        L.hdxo_encode_double.restype = u64
        L.hdxo_hash_timestamp.argtypes = [u32, i64]
        L.hdxo_hash_timestamp.restype = u64
        L.hdxo_hash_value.argtypes = [u32, vp, sz, ctypes.POINTER(ctypes.c_int)]
        L.hdxo_hash_value.restype = u64
        L.hdxo_hash_batch.argtypes = [vp, u32, vp, vp, vp, u64, vp, ctypes.c_int]
        L.hdxo_hash_batch.restype = ctypes.c_int
        L.hdxo_partition.argtypes = [u32, u32, vp, vp, u64]
        L.hdxo_partition.restype = u64
        L.hdxo_lookup_region.argtypes = [u32, u32, vp, vp, vp, vp, vp, u32, u64, vp]
        L.hdxo_lookup_region.restype = None
        L.hdxo_point_leader.argtypes = [u32, vp, ctypes.c_size_t, u32, vp, vp, vp, vp, ctypes.POINTER(ctypes.c_int)]
        L.hdxo_point_leader.restype = u64
        L.hdxo_hash_encoded.argtypes = [vp, u32, vp, vp, vp, vp, vp, vp, u64, vp, vp, vp]
        L.hdxo_index_encode.restype = sz
        L.hdxo_index_encode.argtypes = [u32, vp, sz, vp, ctypes.POINTER(ctypes.c_int)]
        L.hdxo_search_space.restype = ctypes.c_int
        L.hdxo_search_space.argtypes = [u32, vp, vp, vp, vp, vp, vp, vp, u32, vp, vp]
        L.hdxo_search_regions.restype = ctypes.c_int
        L.hdxo_search_regions.argtypes = [u32, u32, vp, vp, vp, vp, vp, u32, vp]
        L.hdxo_hash_encoded.restype = ctypes.c_int64
        _LIB = L
    return _LIB


def ref_lib():
    """oracle/_ref/libref_ordered.so (reference ordered_encoding.cc), or None."""
    global _REF
    if _REF is None:
        path = os.path.join(_HERE, "_ref", "libref_ordered.so")
        if not os.path.exists(path):
            return None
        R = ctypes.CDLL(path)
        R.ref_ordered_encode_int64.argtypes = [ctypes.c_int64]
        R.ref_ordered_encode_int64.restype = ctypes.c_uint64
        R.ref_ordered_encode_double.argtypes = [ctypes.c_double]
        R.ref_ordered_encode_double.restype = ctypes.c_uint64
        _REF = R
    return _REF


def cityhash64(data: bytes) -> int:
    buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    return lib().hdxo_cityhash64(buf, len(data))


def hash_value(type_id: int, data: bytes):
    """hash(hyperdatatype, slice) -> (u64, err)  (common/hash.cc:34-46)."""
    buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    err = ctypes.c_int(0)
    h = lib().hdxo_hash_value(type_id, buf, len(data), ctypes.byref(err))
    return h, err.value


def hash_batch(types, blob, obj_base, attr_len, nthreads=1):
    """Whole-batch oracle over the packed layout.  numpy in, numpy out."""
    types = np.ascontiguousarray(types, dtype=np.uint32)
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    obj_base = np.ascontiguousarray(obj_base, dtype=np.uint64)
    attr_len = np.ascontiguousarray(attr_len, dtype=np.uint32)
    A = len(types)
    n = len(obj_base)
    assert attr_len.size == n * A
    coords = np.zeros(n * A, dtype=np.uint64)
    if blob.size == 0:
        blob = np.zeros(1, dtype=np.uint8)
    err = lib().hdxo_hash_batch(types.ctypes.data, A, blob.ctypes.data,
                                obj_base.ctypes.data, attr_len.ctypes.data, n,
                                coords.ctypes.data, nthreads)
    return coords.reshape(n, A), err


def partition(num_attrs, num_servers):
    """admin/partition.cc: (lower, upper) as (R, num_attrs) uint64 arrays."""
    L = lib()
    R = L.hdxo_partition(num_attrs, num_servers, None, None, 0)
    lower = np.zeros(R * num_attrs, np.uint64)
    upper = np.zeros(R * num_attrs, np.uint64)
    L.hdxo_partition(num_attrs, num_servers, lower.ctypes.data, upper.ctypes.data, R)
    return lower.reshape(R, num_attrs), upper.reshape(R, num_attrs)


def lookup_region(attrs, lower, upper, ids, coords):
    """configuration::lookup_region over every row of coords (n, A)."""
    attrs = np.ascontiguousarray(attrs, np.uint16)
    lower = np.ascontiguousarray(lower, np.uint64)
    upper = np.ascontiguousarray(upper, np.uint64)
    ids = np.ascontiguousarray(ids, np.uint64)
    coords = np.ascontiguousarray(coords, np.uint64)
    n, A = coords.shape
    out = np.zeros(n, np.uint64)
    lib().hdxo_lookup_region(len(attrs), len(ids), attrs.ctypes.data, lower.ctypes.data,
                             upper.ctypes.data, ids.ctypes.data, coords.ctypes.data, A, n,
                             out.ctypes.data)
    return out


def point_leader(key_type, keys, lower0, upper0, leader_vsi, has_replicas):
    """configuration::point_leader (configuration.cc:427-458) for every key of
    `keys` (a list of bytes): (leaders u64 array, aborted bool array — where
    the reference abort()s because no subspace-0 region holds the key)."""
    lower0 = np.ascontiguousarray(lower0, np.uint64).reshape(-1)
    upper0 = np.ascontiguousarray(upper0, np.uint64).reshape(-1)
    vsi = np.ascontiguousarray(leader_vsi, np.uint64)
    rep = np.ascontiguousarray(has_replicas, np.uint8)
    R = len(vsi)
    out = np.zeros(len(keys), np.uint64)
    aborted = np.zeros(len(keys), bool)
    flag = ctypes.c_int(0)
    for i, k in enumerate(keys):
        buf = ctypes.create_string_buffer(bytes(k), max(len(k), 1))
        out[i] = lib().hdxo_point_leader(key_type, buf, len(k), R, lower0.ctypes.data, upper0.ctypes.data,
                                         vsi.ctypes.data, rep.ctypes.data, ctypes.byref(flag))
        aborted[i] = flag.value != 0
    return out, aborted


def hash_encoded(types, keys, key_off, key_len, vals, val_off, val_len):
    """decode_value + hash over stored objects -> (coords (n, A), versions, bad)."""
    types = np.ascontiguousarray(types, np.uint32)
    A = len(types)
    arrs = [np.ascontiguousarray(x, dt) for x, dt in
            ((keys, np.uint8), (key_off, np.uint64), (key_len, np.uint32), (vals, np.uint8),
             (val_off, np.uint64), (val_len, np.uint32))]
    keys, key_off, key_len, vals, val_off, val_len = [a if a.size else np.zeros(1, a.dtype) for a in arrs]
    n = len(arrs[1])
    coords = np.zeros(n * A, np.uint64)
    versions = np.zeros(max(n, 1), np.uint64)
    bad = np.zeros(max(n, 1), np.uint8)
    r = lib().hdxo_hash_encoded(types.ctypes.data, A, keys.ctypes.data, key_off.ctypes.data,
                                key_len.ctypes.data, vals.ctypes.data, val_off.ctypes.data,
                                val_len.ctypes.data, n, coords.ctypes.data, versions.ctypes.data,
                                bad.ctypes.data)
    assert r >= 0
    return coords.reshape(n, A), versions[:n], bad[:n].astype(bool)


def index_encode(type_id: int, data: bytes):
    """Secondary-index key of one value -> (key bytes, err); b"" for other types."""
    buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    out = ctypes.create_string_buffer(16)
    err = ctypes.c_int(0)
    k = lib().hdxo_index_encode(type_id, buf, len(data), out, ctypes.byref(err))
    return out.raw[:k], err.value


class Range(ctypes.Structure):
    """common/range.h after range_searches (layout of hdx_range / hdxo_range)."""
    _fields_ = [("attr", ctypes.c_uint32), ("type", ctypes.c_uint32),
                ("start", ctypes.c_char_p), ("start_len", ctypes.c_uint64),
                ("end", ctypes.c_char_p), ("end_len", ctypes.c_uint64),
                ("has_start", ctypes.c_uint32), ("has_end", ctypes.c_uint32),
                ("invalid", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


def make_ranges(ranges):
    """[(attr, type, start|None, end|None[, invalid])] -> ctypes array of Range."""
    arr = (Range * max(len(ranges), 1))()
    for k, r in enumerate(ranges):
        attr, t, start, end = r[:4]
        arr[k].attr, arr[k].type = attr, t
        arr[k].has_start, arr[k].has_end = start is not None, end is not None
        arr[k].start, arr[k].start_len = (start or b""), len(start or b"")
        arr[k].end, arr[k].end_len = (end or b""), len(end or b"")
        arr[k].invalid = bool(r[4]) if len(r) > 4 else False
    return arr


def search_regions(attrs, lower, upper, ranges, has_replicas=None):
    """lookup_search's region loop for one subspace -> (include u8[R], cleared).
    has_replicas (u8[R] or None = every region has replicas): regions without
    replicas are skipped first (configuration.cc:782-785)."""
    attrs = np.ascontiguousarray(attrs, np.uint16)
    lower = np.ascontiguousarray(lower, np.uint64)
    upper = np.ascontiguousarray(upper, np.uint64)
    R = lower.shape[0] if lower.ndim == 2 else lower.size // max(len(attrs), 1)
    include = np.zeros(max(R, 1), np.uint8)
    arr = make_ranges(ranges)
    rep = None if has_replicas is None else np.ascontiguousarray(has_replicas, np.uint8)
    rc = lib().hdxo_search_regions(len(attrs), R, attrs.ctypes.data, lower.ctypes.data,
                                   upper.ctypes.data, None if rep is None else rep.ctypes.data, arr,
                                   len(ranges), include.ctypes.data)
    if rc < 0:
        raise ValueError("numeric endpoint not 0 or 8 bytes")
    return include[:R], bool(rc)


def search_space(subspaces, ranges, has_replicas=None):
    """lookup_search over subspaces [(attrs, lower, upper), ...] in order ->
    (chosen index or -1, its include mask, cleared); configuration.cc:771-868."""
    T = len(subspaces)
    keep = []
    D = np.array([len(a) for a, _, _ in subspaces] or [0], np.uint32)
    R = np.zeros(max(T, 1), np.uint32)
    P = [(ctypes.c_void_p * max(T, 1))() for _ in range(4)]
    for i, (a, lo, up) in enumerate(subspaces):
        a = np.ascontiguousarray(a, np.uint16)
        lo = np.ascontiguousarray(lo, np.uint64).reshape(-1)
        up = np.ascontiguousarray(up, np.uint64).reshape(-1)
        R[i] = lo.size // max(len(a), 1)
        keep += [a, lo, up]
        P[0][i], P[1][i], P[2][i] = a.ctypes.data, lo.ctypes.data, up.ctypes.data
        if has_replicas is not None and has_replicas[i] is not None:
            r = np.ascontiguousarray(has_replicas[i], np.uint8)
            keep.append(r)
            P[3][i] = r.ctypes.data
    include = np.zeros(max(int(R.max()) if T else 1, 1), np.uint8)
    cleared = ctypes.c_int(0)
    arr = make_ranges(ranges)
    c = lib().hdxo_search_space(T, D.ctypes.data, R.ctypes.data, P[0], P[1], P[2],
                                None if has_replicas is None else P[3], arr, len(ranges),
                                include.ctypes.data, ctypes.byref(cleared))
    if c == -2:
        raise ValueError("numeric endpoint not 0 or 8 bytes")
    return c, (include[:R[c]] if c >= 0 else include[:0]), bool(cleared.value)
