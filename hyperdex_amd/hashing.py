"""Python mirror of the reference hashing interface (common/hash.h:43-55).

    hash(type, value)               -> uint64_t hash(hyperdatatype, const e::slice&)
    hash_key(schema, key)           -> void hash(const schema&, const e::slice& key, uint64_t* h)
    hash_object(schema, key, vals)  -> void hash(const schema&, key, std::vector<e::slice>, uint64_t* hs)

plus the batched GPU path over the packed layout of include/hdxhash.h:

    hash_batch(types, blob, obj_base, attr_len)       device-resident (torch HIP tensors)
    hash_batch_host(types, blob, obj_base, attr_len)  host-resident (numpy), pipelined H2D/D2H
    hash_batch_regions_host(...)                      host-resident, region ids out
    hash_encoded_host(...) / hash_encoded_regions_host(...)
                                                      the reindex sweep from host memory
    hash_batch_device_multi / hash_batch_regions_device_multi
                                                      one shard per device of the set, RCCL gather

All of them run the gfx950 kernels in libhdxhash.so.  Where the reference
asserts (unknown type, mis-sized numeric value) these raise HdxError.
"""
import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import HdxError, check, lib
from .datatypes import Schema


def _u32_array(xs):
    arr = np.ascontiguousarray(np.asarray(xs, dtype=np.uint32))
    return arr


def schema_check(types) -> None:
    t = _u32_array(types)
    check(lib().hdx_schema_check(t.ctypes.data, len(t)))


def hashable(type_id: int) -> bool:
    return bool(lib().hdx_type_hashable(type_id))


def hash(type_id: int, value: bytes) -> int:  # noqa: A001 (mirrors hyperdex::hash)
    out = ctypes.c_uint64(0)
    buf = ctypes.create_string_buffer(bytes(value), max(len(value), 1))
    check(lib().hdx_hash_value(type_id, buf, len(value), ctypes.byref(out)))
    return out.value


def _types_of(sc):
    return sc.types() if isinstance(sc, Schema) else list(sc)


def hash_key(sc, key: bytes) -> int:
    t = _u32_array(_types_of(sc))
    out = ctypes.c_uint64(0)
    buf = ctypes.create_string_buffer(bytes(key), max(len(key), 1))
    check(lib().hdx_hash_key(t.ctypes.data, len(t), buf, len(key), ctypes.byref(out)))
    return out.value


def hash_object(sc, key: bytes, values: Sequence[bytes]):
    t = _u32_array(_types_of(sc))
    A = len(t)
    if len(values) < A - 1:
        raise HdxError(_lib.HDX_E_INVALID, "need %d values, got %d" % (A - 1, len(values)))
    bufs = [ctypes.create_string_buffer(bytes(v), max(len(v), 1)) for v in values[:A - 1]]
    ptrs = (ctypes.c_void_p * max(A - 1, 1))(*[ctypes.addressof(b) for b in bufs])
    lens = (ctypes.c_size_t * max(A - 1, 1))(*[len(v) for v in values[:A - 1]])
    out = (ctypes.c_uint64 * A)()
    kbuf = ctypes.create_string_buffer(bytes(key), max(len(key), 1))
    check(lib().hdx_hash_object(t.ctypes.data, A, kbuf, len(key), ptrs, lens, out))
    return list(out)


def hash_batch(types, blob, obj_base, attr_len, coords=None, status=None, stream=None):
    """Device-resident batch.  blob/obj_base/attr_len/coords are torch tensors on
    a HIP device (any integer dtype of the right width); returns coords (n, A)
    as an int64 tensor holding the uint64 bit patterns.  Asynchronous on
    `stream` (default: torch's current stream)."""
    import torch

    t = _u32_array(types)
    A = len(t)
    n = obj_base.numel()
    _check_packed(blob, obj_base, attr_len, A)
    if coords is None:
        coords = torch.empty((n, A), dtype=torch.int64, device=obj_base.device)
    _check_out(coords, n * A, obj_base.device, "coords")
    _check_status(status, obj_base.device)
    if stream is None:
        stream = torch.cuda.current_stream(obj_base.device)
    handle = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    check(lib().hdx_hash_batch_device(
        t.ctypes.data, A, blob.data_ptr(), obj_base.data_ptr(), attr_len.data_ptr(), n,
        coords.data_ptr(), status.data_ptr() if status is not None else None, handle))
    return coords


def _check_packed(blob, obj_base, attr_len, A):
    """The packed layout's device tensors: u8 blob, u64 bases, u32 lengths (n*A)."""
    n = obj_base.numel()
    assert attr_len.numel() == n * A, "attr_len must hold n*A lengths"
    assert blob.element_size() == 1 and obj_base.element_size() == 8 and attr_len.element_size() == 4, \
        "blob / obj_base / attr_len must have 1 / 8 / 4-byte elements"
    for x in (blob, obj_base, attr_len):
        assert x.is_cuda and x.is_contiguous() and x.device == obj_base.device, "contiguous tensors on one device"


def _check_stored(keys, key_off, key_len, vals, val_off, val_len):
    """Stored objects: u8 keys / values, u64 offsets, u32 lengths, n of each."""
    n = val_off.numel()
    assert key_off.numel() == n and key_len.numel() == n and val_len.numel() == n
    assert keys.element_size() == 1 and vals.element_size() == 1
    assert key_off.element_size() == 8 and val_off.element_size() == 8
    assert key_len.element_size() == 4 and val_len.element_size() == 4
    for x in (keys, key_off, key_len, vals, val_off, val_len):
        assert x.is_cuda and x.is_contiguous() and x.device == val_off.device


def _check_out(x, numel, device, what):
    assert x.is_cuda and x.is_contiguous() and x.element_size() == 8 and x.device == device, \
        "%s must be a contiguous 8-byte tensor on %s" % (what, device)
    assert x.numel() == numel, "%s must hold %d elements, has %d" % (what, numel, x.numel())


def _check_status(status, device):
    if status is not None:
        assert status.is_cuda and status.device == device and status.numel() * status.element_size() >= 4, \
            "status must be a device tensor of at least 4 bytes"


def hash_batch_host(types, blob, obj_base, attr_len, out: Optional[np.ndarray] = None):
    """Host-resident batch (numpy in, numpy (n, A) uint64 out), synchronous."""
    t = _u32_array(types)
    A = len(t)
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    obj_base = np.ascontiguousarray(obj_base, dtype=np.uint64)
    attr_len = np.ascontiguousarray(attr_len, dtype=np.uint32)
    n = len(obj_base)
    assert attr_len.size == n * A
    if out is None:
        out = np.empty((n, A), dtype=np.uint64)
    check(lib().hdx_hash_batch_host(t.ctypes.data, A, blob.ctypes.data if blob.size else None,
                                    blob.size, obj_base.ctypes.data, attr_len.ctypes.data, n,
                                    out.ctypes.data))
    return out


def _handles(tables):
    return (ctypes.c_void_p * max(len(tables), 1))(*[tb.handle.value for tb in tables])


def hash_batch_regions_host(types, blob, obj_base, attr_len, tables, coords: bool = False):
    """hdx_hash_batch_regions_host: host-resident batch -> region ids (T, n)
    uint64 in the RegionTables `tables` (1..4); with coords=True also the
    (n, A) coordinates.  Split over the device set like hash_batch_host."""
    t = _u32_array(types)
    A = len(t)
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    obj_base = np.ascontiguousarray(obj_base, dtype=np.uint64)
    attr_len = np.ascontiguousarray(attr_len, dtype=np.uint32)
    n = len(obj_base)
    assert attr_len.size == n * A
    ids = np.empty((len(tables), n), dtype=np.uint64)
    out = np.empty((n, A), dtype=np.uint64) if coords else None
    check(lib().hdx_hash_batch_regions_host(t.ctypes.data, A, blob.ctypes.data if blob.size else None, blob.size,
                                            obj_base.ctypes.data, attr_len.ctypes.data, n, _handles(tables),
                                            len(tables), ids.ctypes.data, out.ctypes.data if coords else None))
    return (ids, out) if coords else ids


def _stored_host(keys, key_off, key_len, vals, val_off, val_len):
    records = vals is keys  # one store of [key][value] records: keep it one buffer
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    vals = keys if records else np.ascontiguousarray(vals, dtype=np.uint8)
    key_off = np.ascontiguousarray(key_off, dtype=np.uint64)
    key_len = np.ascontiguousarray(key_len, dtype=np.uint32)
    val_off = np.ascontiguousarray(val_off, dtype=np.uint64)
    val_len = np.ascontiguousarray(val_len, dtype=np.uint32)
    n = len(val_off)
    assert len(key_off) == n and len(key_len) == n and len(val_len) == n
    return keys, key_off, key_len, vals, val_off, val_len, n


def hash_encoded_host(types, keys, key_off, key_len, vals, val_off, val_len, versions: bool = False):
    """hdx_hash_encoded_host: the reindex sweep over stored objects in host
    memory (numpy; pass the same array as keys and vals for records
    [key][value] in one store).  Returns coords (n, A) uint64 (and versions (n,)
    with versions=True); raises HdxError (HDX_E_BADENC / HDX_E_BADSIZE) after
    the whole call ran when a value does not decode or a numeric is
    mis-sized — use hash_encoded_host_status to keep the outputs then."""
    coords, vers, st, msg = hash_encoded_host_status(types, keys, key_off, key_len, vals, val_off, val_len)
    if st != _lib.HDX_OK:
        raise HdxError(st, msg)
    return (coords, vers) if versions else coords


def hash_encoded_host_status(types, keys, key_off, key_len, vals, val_off, val_len, tables=()):
    """The same, never raising for undecodable values: (coords, versions,
    status, message), plus region ids (T, n) as a 5th item with `tables`."""
    t = _u32_array(types)
    A = len(t)
    keys, key_off, key_len, vals, val_off, val_len, n = _stored_host(keys, key_off, key_len, vals, val_off, val_len)
    coords = np.empty((n, A), dtype=np.uint64)
    vers = np.empty(n, dtype=np.uint64)
    kp = keys.ctypes.data if keys.size else None
    vp = kp if vals is keys else (vals.ctypes.data if vals.size else None)
    if tables:
        ids = np.empty((len(tables), n), dtype=np.uint64)
        st = lib().hdx_hash_encoded_regions_host(t.ctypes.data, A, kp, keys.size, key_off.ctypes.data,
                                                 key_len.ctypes.data, vp, vals.size, val_off.ctypes.data,
                                                 val_len.ctypes.data, n, _handles(tables), len(tables),
                                                 ids.ctypes.data, coords.ctypes.data, vers.ctypes.data)
    else:
        st = lib().hdx_hash_encoded_host(t.ctypes.data, A, kp, keys.size, key_off.ctypes.data, key_len.ctypes.data,
                                         vp, vals.size, val_off.ctypes.data, val_len.ctypes.data, n,
                                         coords.ctypes.data, vers.ctypes.data)
    msg = ""
    if st != _lib.HDX_OK:
        m = lib().hdx_last_error()
        msg = m.decode() if m else ""
        if st not in (_lib.HDX_E_BADENC, _lib.HDX_E_BADSIZE):
            raise HdxError(st, msg)
    return (coords, vers, st, msg, ids) if tables else (coords, vers, st, msg)


def hash_encoded(types, keys, key_off, key_len, vals, val_off, val_len, coords=None,
                 versions=None, status=None, stream=None):
    """Reindex sweep over stored objects (hdx_hash_encoded_device): values in the
    daemon's on-disk encoding (daemon/datalayer_encodings.cc:139-217) and keys,
    as torch HIP tensors; returns coords (n, A) int64 (uint64 bit patterns)."""
    import torch

    t = _u32_array(types)
    A = len(t)
    n = val_off.numel()
    _check_stored(keys, key_off, key_len, vals, val_off, val_len)
    if coords is None:
        coords = torch.empty((n, A), dtype=torch.int64, device=val_off.device)
    _check_out(coords, n * A, val_off.device, "coords")
    if versions is not None:
        _check_out(versions, n, val_off.device, "versions")
    _check_status(status, val_off.device)
    if stream is None:
        stream = torch.cuda.current_stream(val_off.device)
    handle = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    check(lib().hdx_hash_encoded_device(
        t.ctypes.data, A, keys.data_ptr(), key_off.data_ptr(), key_len.data_ptr(), vals.data_ptr(),
        val_off.data_ptr(), val_len.data_ptr(), n, coords.data_ptr(),
        versions.data_ptr() if versions is not None else None,
        status.data_ptr() if status is not None else None, handle))
    return coords


def hash_encoded_regions(types, keys, key_off, key_len, vals, val_off, val_len, tables, coords=False,
                         versions=None, status=None, stream=None):
    """The sweep with the new regions in the same launch
    (hdx_hash_encoded_regions_device): returns region ids (T, n) int64 for the
    RegionTables `tables` (1..4), and the coordinates too when coords is True
    (or a tensor to fill)."""
    import torch

    t = _u32_array(types)
    A = len(t)
    n = val_off.numel()
    _check_stored(keys, key_off, key_len, vals, val_off, val_len)
    dev = val_off.device
    ids = torch.empty((len(tables), n), dtype=torch.int64, device=dev)
    if coords is True:
        coords = torch.empty((n, A), dtype=torch.int64, device=dev)
    if coords is not None and coords is not False:
        _check_out(coords, n * A, dev, "coords")
    if versions is not None:
        _check_out(versions, n, dev, "versions")
    _check_status(status, dev)
    handles = (ctypes.c_void_p * max(len(tables), 1))(*[tb.handle.value for tb in tables])
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    handle = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    check(lib().hdx_hash_encoded_regions_device(
        t.ctypes.data, A, keys.data_ptr(), key_off.data_ptr(), key_len.data_ptr(), vals.data_ptr(),
        val_off.data_ptr(), val_len.data_ptr(), n, handles, len(tables), ids.data_ptr(),
        coords.data_ptr() if coords is not None and coords is not False else None,
        versions.data_ptr() if versions is not None else None,
        status.data_ptr() if status is not None else None, handle))
    return (ids, coords) if coords is not None and coords is not False else ids


def hash_batch_regions(types, blob, obj_base, attr_len, tables, coords=False, status=None, stream=None):
    """hash_batch fused with the region lookup (hdx_hash_batch_regions_device):
    returns region ids (T, n) int64 for the RegionTables `tables` (1..4) of
    the packed batch, and the coordinates too when coords is True (or a
    tensor to fill)."""
    import torch

    t = _u32_array(types)
    A = len(t)
    n = obj_base.numel()
    _check_packed(blob, obj_base, attr_len, A)
    dev = obj_base.device
    ids = torch.empty((len(tables), n), dtype=torch.int64, device=dev)
    if coords is True:
        coords = torch.empty((n, A), dtype=torch.int64, device=dev)
    if coords is not None and coords is not False:
        _check_out(coords, n * A, dev, "coords")
    _check_status(status, dev)
    handles = (ctypes.c_void_p * max(len(tables), 1))(*[tb.handle.value for tb in tables])
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    handle = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    check(lib().hdx_hash_batch_regions_device(
        t.ctypes.data, A, blob.data_ptr(), obj_base.data_ptr(), attr_len.data_ptr(), n, handles, len(tables),
        ids.data_ptr(), coords.data_ptr() if coords is not None and coords is not False else None,
        status.data_ptr() if status is not None else None, handle))
    return (ids, coords) if coords is not None and coords is not False else ids


def kernel_for(types, n: int):
    """(variant, kernel symbol) hash_batch would launch for this schema and n."""
    t = _u32_array(types)
    name = ctypes.c_char_p()
    v = lib().hdxdbg_kernel_for(t.ctypes.data, len(t), n, ctypes.byref(name))
    return v, (name.value or b"").decode()


# ---- the device set (hdx_init_mask; include/hdxhash.h "multi-device") ------

def init_mask(mask: int) -> None:
    """hdx_init_mask: the process's device set (bit d = HIP ordinal d).  After
    it hash_batch_host splits every batch over the set's devices, and
    hash_batch_device_multi takes one shard per device."""
    check(lib().hdx_init_mask(mask))


def device_set():
    """The device set's HIP ordinals (empty before init_mask)."""
    buf = (ctypes.c_int * 64)()
    k = lib().hdx_device_set(buf, 64)
    return list(buf[:k])


def shutdown() -> None:
    """hdx_shutdown: tear the device set down and free every thread's scratch."""
    check(lib().hdx_shutdown())


def shard_ranges(attr_len, attrs_sz: int, n: int, world: int, equal_count_tol: float = 0.0):
    """hdx_shard_ranges (the C++ cut rule): (first, count) per shard, the
    same cuts as hyperdex_amd.dist.shard_ranges(n, world, per-object bytes)."""
    first = np.zeros(world + 1, dtype=np.uint64)
    if attr_len is None:
        check(lib().hdx_shard_ranges(None, attrs_sz, n, world, equal_count_tol, first.ctypes.data))
    else:
        lens = np.ascontiguousarray(attr_len, dtype=np.uint32)
        assert lens.size == n * attrs_sz
        check(lib().hdx_shard_ranges(lens.ctypes.data, attrs_sz, n, world, equal_count_tol, first.ctypes.data))
    f = [int(x) for x in first]
    return [(f[k], f[k + 1] - f[k]) for k in range(world)]


def hash_batch_device_multi(types, shards, gather: bool = True, coords=None):
    """hdx_hash_batch_device_multi: shards[k] = (blob, obj_base, attr_len) torch
    tensors on the k-th device of the set (status tensors optional as a 4th
    item).  gather: returns one (N, A) int64 matrix per device, every device
    holding all rows (RCCL over the set); else each shard's own (n_k, A)
    coordinates.  `coords` may pass those output tensors in."""
    import torch

    t = _u32_array(types)
    A = len(t)
    counts = [int(s[1].numel()) for s in shards]
    N = sum(counts)
    outs = []
    arr = (_lib.Shard * max(len(shards), 1))()
    for k, s in enumerate(shards):
        blob, base, lens = s[0], s[1], s[2]
        status = s[3] if len(s) > 3 else None
        _check_packed(blob, base, lens, A)
        rows = N if gather else counts[k]
        out = coords[k] if coords is not None else torch.empty((rows, A), dtype=torch.int64, device=base.device)
        _check_out(out, rows * A, base.device, "coords")
        _check_status(status, base.device)
        outs.append(out)
        arr[k] = _lib.Shard(blob.data_ptr(), base.data_ptr(), lens.data_ptr(), counts[k], out.data_ptr(),
                            status.data_ptr() if status is not None else None)
    # the library's streams run the work: order it after torch's current streams
    for s in shards:
        torch.cuda.current_stream(s[1].device).synchronize()
    check(lib().hdx_hash_batch_device_multi(t.ctypes.data, A, arr, len(shards), 1 if gather else 0))
    return outs


def hash_batch_regions_device_multi(types, shards, tables, gather: bool = True, coords: bool = False):
    """hdx_hash_batch_regions_device_multi: shards[k] = (blob, obj_base,
    attr_len[, status]) on the k-th device of the set; returns one region-id
    tensor per device — (T, N) with gather (every device holds every object's
    ids: only the ids cross the fabric), else (T, n_k) — and, with coords=True,
    each shard's own (n_k, A) coordinates as a second list."""
    import torch

    t = _u32_array(types)
    A = len(t)
    T = len(tables)
    counts = [int(s[1].numel()) for s in shards]
    N = sum(counts)
    ids_out, coord_out = [], []
    arr = (_lib.RegionShard * max(len(shards), 1))()
    for k, s in enumerate(shards):
        blob, base, lens = s[0], s[1], s[2]
        status = s[3] if len(s) > 3 else None
        _check_packed(blob, base, lens, A)
        _check_status(status, base.device)
        ids = torch.empty((T, N if gather else counts[k]), dtype=torch.int64, device=base.device)
        c = torch.empty((counts[k], A), dtype=torch.int64, device=base.device) if coords else None
        ids_out.append(ids)
        coord_out.append(c)
        arr[k] = _lib.RegionShard(blob.data_ptr(), base.data_ptr(), lens.data_ptr(), counts[k], ids.data_ptr(),
                                  c.data_ptr() if c is not None else None,
                                  status.data_ptr() if status is not None else None)
    for s in shards:
        torch.cuda.current_stream(s[1].device).synchronize()
    check(lib().hdx_hash_batch_regions_device_multi(t.ctypes.data, A, arr, len(shards), _handles(tables), T,
                                                    1 if gather else 0))
    return (ids_out, coord_out) if coords else ids_out
