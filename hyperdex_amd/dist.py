"""Multi-GPU batches: shard objects across ranks, hash locally, gather coordinates.

Objects are independent (common/hash.cc:56-68 keeps no cross-object state),
so a batch splits into contiguous object ranges, one per rank (one process
per GPU), balanced by payload bytes.  Each rank hashes its range
with the gfx950 kernel straight into its rows of the full (n, A) coordinate
matrix; no collective is needed for that.  The only exchange is the optional
all-gather of those rows (torch.distributed: RCCL over xGMI on the "nccl"
backend, gloo on CPU), in place in the same matrix, reported separately from
the hash phase by bench.py (config 4).
"""
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np


def shard_ranges(n: int, world: int, obj_sizes=None) -> List[Tuple[int, int]]:
    """Contiguous (first, count) object ranges, one per rank.

    Without sizes: counts differ by at most one.  With per-object payload
    sizes (numpy array, or a torch tensor — then the prefix sum and the
    search run on its device): rank k starts at the first object whose byte
    prefix reaches k/world of the total.  Both forms give the same cuts."""
    if world < 1:
        raise ValueError("world must be >= 1")
    if obj_sizes is None:
        cuts = [n * k // world for k in range(world + 1)]
    elif hasattr(obj_sizes, "is_cuda"):  # torch tensor
        import torch
        assert obj_sizes.numel() == n
        csum = torch.zeros(n + 1, dtype=torch.float64, device=obj_sizes.device)
        if n:
            torch.cumsum(obj_sizes.to(torch.float64), dim=0, out=csum[1:])
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
        cuts = [0]
        for k in range(1, world):
            c = int(np.searchsorted(csum, csum[-1] * k / world, side="left"))
            cuts.append(min(max(c, cuts[-1]), n))
        cuts.append(n)
    return [(cuts[k], cuts[k + 1] - cuts[k]) for k in range(world)]


def rank_rows(out, counts: Sequence[int], rank: int):
    """This rank's rows of the full (sum(counts), A) coordinate matrix (a view)."""
    first = int(sum(counts[:rank]))
    return out[first:first + int(counts[rank])]


def allgather_coords(local, counts: Sequence[int], group=None, out=None):
    """Every rank's (count_r, A) coordinate block, in rank order, in `out`
    (allocated when None) — no padding and no concatenation copy.

    `local` may already be this rank's rows of `out` (rank_rows); otherwise it
    is copied there.  Equal counts on RCCL/NCCL: one in-place
    all_gather_into_tensor.  Unequal counts (byte-balanced shards) or gloo:
    one broadcast per rank into that rank's rows."""
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
    if mine.data_ptr() != local.data_ptr():
        mine.copy_(local)
    if dist.get_backend(group) == "nccl" and len(set(counts)) == 1:
        dist.all_gather_into_tensor(out, mine, group=group)  # in place: mine == out + rank * count
        return out
    first = 0
    for r, c in enumerate(counts):
        if c:
            src = dist.get_global_rank(group, r) if group is not None else r
            dist.broadcast(out[first:first + c], src=src, group=group)
        first += c
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
