"""Multi-GPU batches: shard objects across ranks, hash locally, gather coordinates.

Objects are independent (common/hash.cc:56-68 keeps no cross-object state),
so a batch splits into contiguous object ranges, one per rank (one process
per GPU), balanced by payload bytes.  Each rank hashes its range
with the gfx950 kernel; no collective is needed for that.  The only exchange
is the optional all-gather of the n x A coordinate matrix (torch.distributed:
RCCL over xGMI on the "nccl" backend, gloo on CPU), reported separately from
the hash phase by bench.py.
"""
from typing import List, Optional, Sequence, Tuple

import numpy as np


def shard_ranges(n: int, world: int, obj_sizes: Optional[Sequence[int]] = None) -> List[Tuple[int, int]]:
    """Contiguous (first, count) object ranges, one per rank.

    Without sizes: counts differ by at most one.  With per-object payload
    sizes: rank k starts at the first object whose byte prefix reaches
    k/world of the total."""
    if world < 1:
        raise ValueError("world must be >= 1")
    if obj_sizes is None:
        cuts = [n * k // world for k in range(world + 1)]
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


def allgather_coords(local, counts: Sequence[int], group=None):
    """Concatenate every rank's (count_r, A) coordinate block in rank order.

    RCCL/NCCL: one all_gather_into_tensor over a buffer padded to the largest
    block; gloo: all_gather of the padded blocks."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    assert len(counts) == world
    A = local.shape[1]
    m = max(counts)
    if local.shape[0] < m:
        pad = torch.zeros((m - local.shape[0], A), dtype=local.dtype, device=local.device)
        local = torch.cat([local, pad])
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world * m, A), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
        blocks = out.view(world, m, A)
    else:
        parts = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(parts, local.contiguous(), group=group)
        blocks = torch.stack(parts)
    return torch.cat([blocks[r, :counts[r]] for r in range(world)])


def hash_sharded(types, blob, obj_base, attr_len, counts: Sequence[int], group=None,
                 gather: bool = True, stream=None):
    """Hash this rank's shard (device tensors) and optionally gather all shards.

    `counts` holds every rank's object count (shard_ranges).  Returns the local
    (count, A) coordinates, or the full (sum(counts), A) matrix if gather."""
    from .hashing import hash_batch

    coords = hash_batch(types, blob, obj_base, attr_len, stream=stream)
    if not gather:
        return coords
    return allgather_coords(coords, counts, group)
