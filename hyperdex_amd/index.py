"""Secondary-index keys and search pruning on the GPU.

index_encode   index_encoding_{int64,timestamp,float}::encode
               (daemon/index_int64.cc:76-79, index_timestamp.cc:79-82,
               index_float.cc:75-90) over a column of values in HBM.
search_regions the region test of configuration::lookup_search
               (common/configuration.cc:736-858) for one subspace's table.
"""
import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np

from ._lib import check, lib
from .regions import RegionTable


def index_key_size(type_id: int) -> int:
    """8 for INT64/TIMESTAMP_*, 16 for FLOAT, 0 otherwise."""
    return int(lib().hdx_index_key_size(type_id))


def index_encode(type_id: int, blob, off, length, out=None, status=None, stream=None):
    """Index keys of n values (value i = blob[off[i] : off[i] + length[i]]), all
    HIP tensors; returns a (n, key_size) uint8 tensor."""
    import torch

    size = index_key_size(type_id)
    n = off.numel()
    assert length.numel() == n and off.element_size() == 8 and length.element_size() == 4
    for x in (blob, off, length):
        assert x.is_cuda and x.is_contiguous()
    if out is None:
        out = torch.empty((n, max(size, 1)), dtype=torch.uint8, device=off.device)
    if stream is None:
        stream = torch.cuda.current_stream(off.device)
    handle = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    check(lib().hdx_index_encode_device(type_id, blob.data_ptr(), off.data_ptr(), length.data_ptr(), n,
                                        out.data_ptr(), status.data_ptr() if status is not None else None,
                                        handle))
    return out


class Range(ctypes.Structure):
    """hdx_range: one range of a search after range_searches()
    (common/range.h:40-55): inclusive, start/end optional."""
    _fields_ = [("attr", ctypes.c_uint32), ("type", ctypes.c_uint32),
                ("start", ctypes.c_char_p), ("start_len", ctypes.c_uint64),
                ("end", ctypes.c_char_p), ("end_len", ctypes.c_uint64),
                ("has_start", ctypes.c_uint32), ("has_end", ctypes.c_uint32),
                ("invalid", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


def _ranges(ranges: Sequence[tuple]):
    arr = (Range * max(len(ranges), 1))()
    for k, r in enumerate(ranges):
        attr, t, start, end = r[:4]
        arr[k].attr, arr[k].type = attr, t
        arr[k].has_start, arr[k].has_end = start is not None, end is not None
        arr[k].start, arr[k].start_len = (start or b""), len(start or b"")
        arr[k].end, arr[k].end_len = (end or b""), len(end or b"")
        arr[k].invalid = bool(r[4]) if len(r) > 4 else False
    return arr


def search_regions(table: RegionTable, ranges: Sequence[tuple],
                   has_replicas=None) -> Tuple[np.ndarray, bool]:
    """ranges: [(attr, hyperdatatype, start bytes | None, end bytes | None[, invalid])].
    has_replicas: u8[R] (0 = the region has no replicas and is skipped, as
    configuration.cc:782-785 does) or None (all have).  Returns (include u8[R],
    cleared): include[r] = 0 when region r is skipped or a range rules it out;
    cleared when the reference returns an empty server list."""
    R = len(table.ids)
    include = np.zeros(max(R, 1), np.uint8)
    cleared = ctypes.c_int(0)
    arr = _ranges(ranges)
    rep = None
    if has_replicas is not None:
        rep = np.ascontiguousarray(has_replicas, np.uint8)
        assert rep.size == R, "has_replicas must hold one flag per region"
    check(lib().hdx_search_regions(table.handle, arr, len(ranges), None if rep is None else rep.ctypes.data,
                                   include.ctypes.data, ctypes.byref(cleared)))
    return include[:R], bool(cleared.value)


def search_space(tables: Sequence[RegionTable], ranges: Sequence[tuple],
                 has_replicas=None) -> Tuple[int, np.ndarray, bool]:
    """configuration::lookup_search over a space's subspaces (tables in the
    space's order; hdx_search_space).  has_replicas: None or one u8[R] array
    (or None) per table.  Returns (chosen subspace index or -1, its include
    mask u8[R], cleared)."""
    T = len(tables)
    handles = (ctypes.c_void_p * max(T, 1))(*[t.handle for t in tables])
    rmax = max([len(t.ids) for t in tables] + [1])
    include = np.zeros(rmax, np.uint8)
    reps, keep = None, []
    if has_replicas is not None:
        assert len(has_replicas) == T
        reps = (ctypes.c_void_p * max(T, 1))()
        for i, r in enumerate(has_replicas):
            if r is not None:
                a = np.ascontiguousarray(r, np.uint8)
                assert a.size == len(tables[i].ids), "has_replicas[%d] must hold one flag per region" % i
                keep.append(a)
                reps[i] = a.ctypes.data
    chosen, servers, cleared = ctypes.c_int32(-1), ctypes.c_uint32(0), ctypes.c_int(0)
    arr = _ranges(ranges)
    check(lib().hdx_search_space(handles, T, arr, len(ranges), reps, ctypes.byref(chosen), include.ctypes.data,
                                 ctypes.byref(servers), ctypes.byref(cleared)))
    c = chosen.value
    mask = include[:len(tables[c].ids)] if c >= 0 else include[:0]
    assert c < 0 or int(mask.sum()) == servers.value
    return c, mask, bool(cleared.value)
