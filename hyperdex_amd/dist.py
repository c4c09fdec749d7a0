"""Multi-GPU batches: shard objects across ranks, hash locally, gather coordinates.

Objects are independent (common/hash.cc:56-68 keeps no cross-object state),
so a batch splits into contiguous object ranges, one per rank (one process
per GPU), balanced by payload bytes.  Each rank hashes its range
with the gfx950 kernel straight into its rows of the full (n, A) coordinate
matrix; no collective is needed for that.  The only exchange is the optional
all-gather of those rows (torch.distributed: RCCL over xGMI on the "nccl"
backend, gloo on CPU), in place in the same matrix, reported separately from
the hash phase by bench.py (config 4): one all_gather_into_tensor per
gather whatever the counts.
"""
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np


def shard_ranges(n: int, world: int, obj_sizes=None,
                 equal_count_tol: float = 0.0) -> List[Tuple[int, int]]:
    """Contiguous (first, count) object ranges, one per rank.

    Without sizes: counts differ by at most one.  With per-object payload
    sizes (numpy array, or a torch tensor — then the prefix sum and the
    search run on its device): rank k starts at the first object whose byte
    prefix reaches k/world of the total.  Both forms give the same cuts.

    equal_count_tol > 0: take the equal-count cuts instead whenever no rank's
    bytes then differ from the mean share by more than that fraction (so the
    gather is one in-place all-gather with no padding; at config 4's 100 M
    objects the equal-count imbalance is ~1e-4)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    even = [n * k // world for k in range(world + 1)]
    if obj_sizes is None:
        cuts = even
    elif hasattr(obj_sizes, "is_cuda"):  # torch tensor
        import torch
        assert obj_sizes.numel() == n
        csum = torch.zeros(n + 1, dtype=torch.float64, device=obj_sizes.device)
        if n:
            torch.cumsum(obj_sizes.to(torch.float64), dim=0, out=csum[1:])
        if equal_count_tol > 0 and _within(csum[even].tolist(), world, equal_count_tol):
            cuts = even
        else:
            total = float(csum[-1].item())
            targets = torch.tensor([total * k / world for k in range(1, world)], dtype=torch.float64,
                                   device=obj_sizes.device)
            found = torch.searchsorted(csum, targets, right=False).tolist() if world > 1 else []
            cuts = [0]
            for c in found:
                cuts.append(min(max(int(c), cuts[-1]), n))
            cuts.append(n)
    else:
        sizes = np.asarray(obj_sizes, dtype=np.float64)
        assert len(sizes) == n
        csum = np.concatenate([[0.0], np.cumsum(sizes)])
        if equal_count_tol > 0 and _within(csum[even].tolist(), world, equal_count_tol):
            cuts = even
        else:
            cuts = [0]
            for k in range(1, world):
                c = int(np.searchsorted(csum, csum[-1] * k / world, side="left"))
                cuts.append(min(max(c, cuts[-1]), n))
            cuts.append(n)
    return [(cuts[k], cuts[k + 1] - cuts[k]) for k in range(world)]


def _within(prefix_at_cuts, world, tol):
    """True if every shard's bytes are within tol of the mean share."""
    total = prefix_at_cuts[-1]
    if total <= 0:
        return True
    share = total / world
    return all(abs((b - a) - share) <= tol * share for a, b in zip(prefix_at_cuts[:-1], prefix_at_cuts[1:]))


def byte_imbalance(ranges, obj_sizes) -> float:
    """max over ranks of |shard bytes - mean share| / mean share."""
    sizes = np.asarray(obj_sizes.cpu() if hasattr(obj_sizes, "is_cuda") else obj_sizes, dtype=np.float64)
    per = [float(sizes[f:f + c].sum()) for f, c in ranges]
    share = sum(per) / max(len(per), 1)
    return max(abs(p - share) for p in per) / share if share else 0.0


def rank_rows(out, counts: Sequence[int], rank: int):
    """This rank's rows of the full (sum(counts), A) coordinate matrix (a view)."""
    first = int(sum(counts[:rank]))
    return out[first:first + int(counts[rank])]


def gather_form(counts: Sequence[int]) -> str:
    """Which single collective allgather_coords issues for these counts."""
    return "in_place" if len(set(int(c) for c in counts)) <= 1 else "padded"


def allgather_coords(local, counts: Sequence[int], group=None, out=None):
    """Every rank's (count_r, A) coordinate block, in rank order, in `out`
    (allocated when None), with exactly ONE collective per call
    (all_gather_into_tensor: RCCL over xGMI on "nccl", gloo on CPU).

    `local` may already be this rank's rows of `out` (rank_rows); otherwise it
    is copied there.  Equal counts: the all-gather runs in place in `out`
    (this rank's rows are its input), no padding, no copy.  Unequal counts
    (byte-balanced shards): every block is padded to the largest count in one
    staging matrix, gathered there, and its rows copied into `out`.

    Memory: the unequal form allocates that staging matrix (world *
    max(counts) * A elements) beside `out`, roughly doubling the gather's
    device memory (config 4: +13.6 GB); shard_ranges(..., equal_count_tol)
    avoids it whenever equal counts stay within the tolerance, and the
    C-ABI's hdx_hash_batch_device_multi gathers unequal counts with grouped
    in-place broadcasts and no staging."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    assert len(counts) == world and local.shape[0] == counts[rank]
    A = local.shape[1]
    if out is None:
        out = torch.empty((int(sum(counts)), A), dtype=local.dtype, device=local.device)
    assert out.shape == (int(sum(counts)), A) and out.is_contiguous()
    mine = rank_rows(out, counts, rank)
    if gather_form(counts) == "in_place":
        if mine.data_ptr() != local.data_ptr():
            mine.copy_(local)
        dist.all_gather_into_tensor(out, mine, group=group)  # in place: mine == out + rank * count
        return out
    cmax = int(max(counts))
    staging = torch.empty((world * cmax, A), dtype=local.dtype, device=local.device)
    slot = staging[rank * cmax:(rank + 1) * cmax]
    slot[:counts[rank]].copy_(local)
    dist.all_gather_into_tensor(staging, slot, group=group)
    first = 0
    for r, c in enumerate(counts):
        if r != rank or mine.data_ptr() != local.data_ptr():
            out[first:first + c].copy_(staging[r * cmax:r * cmax + c])
        first += c
    del staging
    return out


def hash_sharded(types, blob, obj_base, attr_len, counts: Sequence[int], group=None,
                 gather: bool = True, stream=None, out=None,
                 hash_fn: Optional[Callable] = None):
    """Hash this rank's shard (device tensors) and optionally gather all shards.

    `counts` holds every rank's object count (shard_ranges).  With gather (or
    an `out` given), the shard is hashed straight into this rank's rows of
    the full (sum(counts), A) matrix and the all-gather fills the rest in
    place; returns that matrix, else the local (count, A) coordinates.
    hash_fn(types, blob, obj_base, attr_len, coords) defaults to the gfx950
    kernel (hashing.hash_batch); the CPU tests pass their CPU checker."""
    import torch
    import torch.distributed as dist

    from .hashing import hash_batch

    if hash_fn is None:
        def hash_fn(t, b, o, l, coords):
            hash_batch(t, b, o, l, coords=coords, stream=stream)
    A = len(types)
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if out is None and gather:
        out = torch.empty((int(sum(counts)), A), dtype=torch.int64, device=obj_base.device)
    local = rank_rows(out, counts, rank) if out is not None else \
        torch.empty((obj_base.numel(), A), dtype=torch.int64, device=obj_base.device)
    hash_fn(types, blob, obj_base, attr_len, local)
    if not gather:
        return out if out is not None else local
    return allgather_coords(local, counts, group, out=out)
