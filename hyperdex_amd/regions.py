"""Coordinates -> region ids on the GPU.

Mirror of configuration::lookup_region (common/configuration.cc:698-735) and
the region step of point_leader (:427-497): the first region of a subspace
whose box holds the object's coordinates, else region_id() = 0.  Region
boxes come from admin/partition.cc via the coordinator and are input here.
"""
import ctypes

import numpy as np

from ._lib import check, lib


class RegionTable:
    """A subspace's regions on the device (common/hyperspace.h:99-137).

    attrs: the subspace's attribute indices (subspace.attrs); lower/upper:
    (R, D) boxes; ids: (R,) region ids."""

    def __init__(self, attrs, lower, upper, ids):
        self.attrs = np.ascontiguousarray(attrs, np.uint16)
        D = len(self.attrs)
        self.lower = np.ascontiguousarray(lower, np.uint64).reshape(-1, D)
        self.upper = np.ascontiguousarray(upper, np.uint64).reshape(-1, D)
        self.ids = np.ascontiguousarray(ids, np.uint64)
        R = len(self.ids)
        assert self.lower.shape == (R, D) and self.upper.shape == (R, D)
        h = ctypes.c_void_p()
        self._lib = lib()  # destroyed by the library that created it
        check(self._lib.hdx_region_table_create(D, R, self.attrs.ctypes.data, self.lower.ctypes.data,
                                            self.upper.ctypes.data, self.ids.ctypes.data,
                                            ctypes.byref(h)))
        self._h = h

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.hdx_region_table_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def lookup_region(table: RegionTable, coords, out=None, stream=None):
    """coords: (n, A) int64 HIP tensor of coordinates; returns (n,) int64 region ids."""
    import torch

    n, A = coords.shape
    assert coords.is_cuda and coords.is_contiguous() and coords.element_size() == 8
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=coords.device)
    if stream is None:
        stream = torch.cuda.current_stream(coords.device)
    handle = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    check(lib().hdx_lookup_region_device(table.handle, coords.data_ptr(), A, n, out.data_ptr(), handle))
    return out
