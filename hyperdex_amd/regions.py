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


class PointLeaderAbort(RuntimeError):
    """A key no subspace-0 region holds: configuration::point_leader abort()s
    there (common/configuration.cc:453, :490)."""


class PointLeaders:
    """configuration::point_leader (common/configuration.cc:427-458; the
    region_id overload :460-497 runs the same scan) for batches of keys.

    The reference hashes the key alone (hash(sc, key, &h), hash.cc:48-54),
    takes the FIRST subspace-0 region in table order with lower_coord[0] <=
    h <= upper_coord[0], and returns its first replica's virtual server
    (replicas[0].vsi), or virtual_server_id() == 0 when that region has no
    replicas.  Here the key batch goes through ONE fused launch
    (hdx_hash_batch_regions_device, key-only schema) with two tables over the
    same boxes: `leader` (ids = replicas[0].vsi, 0 for a region without
    replicas) and `where` (ids = position + 1, never 0).  A 0 in `where` is
    the reference's abort(); it raises PointLeaderAbort naming the first such
    key instead of ending the process.

    lower0 / upper0: (R,) the subspace-0 boxes in the configuration's order;
    leader_vsi: (R,) replicas[0].vsi; has_replicas: (R,) bool."""

    def __init__(self, lower0, upper0, leader_vsi, has_replicas):
        lower0 = np.ascontiguousarray(lower0, np.uint64).reshape(-1, 1)
        upper0 = np.ascontiguousarray(upper0, np.uint64).reshape(-1, 1)
        R = lower0.shape[0]
        vsi = np.where(np.asarray(has_replicas, bool), np.asarray(leader_vsi, np.uint64), np.uint64(0))
        self.leader = RegionTable([0], lower0, upper0, vsi.astype(np.uint64))
        self.where = RegionTable([0], lower0, upper0, np.arange(1, R + 1, dtype=np.uint64))

    def close(self):
        self.leader.close()
        self.where.close()

    def leaders(self, key_type: int, blob, key_base, key_len, stream=None, check: bool = True):
        """Keys packed as a one-attribute batch (blob, key_base[n], key_len[n]
        on the device) -> ((n,) leader vsi, (n,) subspace-0 region position +
        1), int64 on the device; with check, a key no region holds (position
        0) raises PointLeaderAbort."""
        from .hashing import hash_batch_regions
        ids = hash_batch_regions([key_type], blob, key_base, key_len, [self.leader, self.where], stream=stream)
        if check:
            miss = (ids[1] == 0).nonzero()
            if miss.numel():
                raise PointLeaderAbort("key %d: no subspace-0 region holds its coordinate "
                                       "(configuration::point_leader abort()s)" % int(miss[0, 0]))
        return ids[0], ids[1]
