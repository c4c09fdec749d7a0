"""Daemon batching shim (hdx_batcher_*) from Python.

Mirrors the call key_state::hash_objects makes (daemon/key_state.cc:1455-1543):
hash one whole object and look it up in the space's subspaces, from any
number of threads at once; the library hashes small objects on the calling
thread and coalesces the rest into device batches.  ctypes releases the GIL for the call, so Python threads do overlap.
"""
import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ._lib import check, lib
from .regions import RegionTable


class _Config(ctypes.Structure):
    _fields_ = [("max_objects", ctypes.c_uint32), ("max_delay_us", ctypes.c_uint32),
                ("max_bytes", ctypes.c_uint64), ("slots", ctypes.c_uint32),
                ("device", ctypes.c_int32), ("tables", ctypes.c_void_p),
                ("ntables", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("host_max_bytes", ctypes.c_uint64)]


class _Stats(ctypes.Structure):
    _fields_ = [("objects", ctypes.c_uint64), ("batches", ctypes.c_uint64),
                ("full_batches", ctypes.c_uint64), ("direct", ctypes.c_uint64),
                ("host", ctypes.c_uint64)]


class Batcher:
    """One per space: types = the schema's attribute types (attr 0 = key);
    tables = the subspaces every object is looked up in (RegionTable).
    Objects up to host_max_bytes (0: every object) are hashed on the calling
    thread; device_only ships every object to the GPU."""

    def __init__(self, types: Sequence[int], tables: Sequence[RegionTable] = (),
                 max_objects: int = 0, max_delay_us: int = 0, max_bytes: int = 0,
                 slots: int = 0, device: int = -1, stage_device: bool = False,
                 device_only: bool = False, host_max_bytes: int = 0):
        self.types = np.ascontiguousarray(np.asarray(types, np.uint32))
        self.A = len(self.types)
        self._tables = list(tables)  # keep the handles alive
        self._handles = (ctypes.c_void_p * max(len(tables), 1))(*[t.handle.value for t in tables])
        cfg = _Config(max_objects, max_delay_us, max_bytes, slots, device,
                      ctypes.cast(self._handles, ctypes.c_void_p) if tables else None, len(tables),
                      (1 if stage_device else 0) | (2 if device_only else 0), host_max_bytes)
        h = ctypes.c_void_p()
        check(lib().hdx_batcher_create(self.types.ctypes.data, self.A, ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h

    def hash_object(self, key: bytes, values: Sequence[bytes]) -> Tuple[List[int], List[int]]:
        """(coords[A], region ids[len(tables)]) of one object."""
        A = self.A
        assert len(values) >= A - 1
        vals = [bytes(v) for v in values[:A - 1]]
        ptrs = (ctypes.c_char_p * max(A - 1, 1))(*vals)
        lens = (ctypes.c_size_t * max(A - 1, 1))(*[len(v) for v in vals])
        hs = (ctypes.c_uint64 * A)()
        rid = (ctypes.c_uint64 * max(len(self._tables), 1))()
        check(lib().hdx_batcher_hash_object(self._h, bytes(key), len(key), ptrs, lens, hs, rid))
        return list(hs), list(rid)[:len(self._tables)]

    def stats(self) -> dict:
        s = _Stats()
        check(lib().hdx_batcher_get_stats(self._h, ctypes.byref(s)))
        return {f: getattr(s, f) for f, _ in _Stats._fields_}

    def close(self):
        if getattr(self, "_h", None):
            lib().hdx_batcher_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
