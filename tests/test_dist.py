"""Sharded batches on world_size 2 and 3 (gloo, CPU): shard_ranges +
hash_sharded + allgather_coords — the code path bench.py's config 4 runs
(byte-balanced shards, each rank hashing straight into its rows of the full
coordinate matrix, the all-gather filling the rest in place).

The per-shard coordinates come from the oracle here (no GPU on this host);
the GPU path runs the same functions over RCCL in bench.py --gpus N."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hyperdex_amd import dist as hdist
from hyperdex_amd import synth


def test_shard_ranges_even():
    for n in (0, 1, 7, 64, 1000):
        for world in (1, 2, 3, 8):
            r = hdist.shard_ranges(n, world)
            assert [c for _, c in r] and sum(c for _, c in r) == n
            assert r[0][0] == 0 and all(r[k][0] + r[k][1] == r[k + 1][0] for k in range(world - 1))
            assert max(c for _, c in r) - min(c for _, c in r) <= 1


def test_shard_ranges_byte_balanced():
    rng = np.random.default_rng(2)
    sizes = rng.integers(1, 2000, 5000)
    for world in (2, 4, 8):
        r = hdist.shard_ranges(len(sizes), world, sizes)
        assert sum(c for _, c in r) == len(sizes)
        per = [sizes[f:f + c].sum() for f, c in r]
        assert max(per) - min(per) <= 2 * sizes.max()


def test_shard_ranges_torch_matches_numpy():
    """bench.py computes the byte-balanced cuts on the device (torch); they
    equal the host form's."""
    rng = np.random.default_rng(5)
    for n in (0, 1, 17, 5000):
        sizes = rng.integers(0, 3000, n)
        for world in (1, 2, 3, 8):
            assert hdist.shard_ranges(n, world, torch.from_numpy(sizes)) == hdist.shard_ranges(n, world, sizes)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_ranges_equal_count_tolerance():
    """Equal counts whenever every rank stays within the tolerance of its byte
    share (the single in-place all-gather), byte-balanced cuts otherwise."""
    rng = np.random.default_rng(3)
    sizes = rng.integers(0, 196, 200_000) + 64
    for world in (2, 3, 8):
        even = hdist.shard_ranges(len(sizes), world)
        got = hdist.shard_ranges(len(sizes), world, sizes, equal_count_tol=1e-2)
        assert got == even and hdist.byte_imbalance(got, sizes) <= 1e-2
        assert hdist.shard_ranges(len(sizes), world, torch.from_numpy(sizes), equal_count_tol=1e-2) == even
    skew = np.concatenate([np.full(1000, 10), np.full(1000, 1000)])
    got = hdist.shard_ranges(len(skew), 2, skew, equal_count_tol=1e-3)
    assert got == hdist.shard_ranges(len(skew), 2, skew) and got != hdist.shard_ranges(len(skew), 2)
    assert hdist.gather_form([5, 5]) == "in_place" and hdist.gather_form([5, 6]) == "padded"


class _Count:
    """Counts torch.distributed collectives issued while active."""
    NAMES = ("all_gather_into_tensor", "all_gather", "broadcast", "all_to_all_single",
             "batch_isend_irecv", "send", "recv", "isend", "irecv")

    def __enter__(self):
        self.n, self.saved = 0, {k: getattr(dist, k) for k in self.NAMES}
        for k, fn in self.saved.items():
            def wrap(*a, _fn=fn, **kw):
                self.n += 1
                return _fn(*a, **kw)
            setattr(dist, k, wrap)
        return self

    def __exit__(self, *exc):
        for k, fn in self.saved.items():
            setattr(dist, k, fn)


def _worker(rank, world, port, ret):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    ok = True
    # config 4's gather is ONE collective for equal and for near-equal counts
    for counts in ([40] * world, [40 + (r % 2) for r in range(world)], [1] + [0] * (world - 1)):
        out = torch.full((sum(counts), 3), -1, dtype=torch.int64)
        first = sum(counts[:rank])
        mine = hdist.rank_rows(out, counts, rank)
        mine.copy_(torch.arange(first, first + counts[rank])[:, None].expand(counts[rank], 3))
        with _Count() as c:
            got = hdist.allgather_coords(mine, counts, out=out)
        ok &= c.n == 1 and got.data_ptr() == out.data_ptr()
        ok &= bool(torch.equal(out, torch.arange(sum(counts))[:, None].expand(sum(counts), 3)))
    for n in (301, 64):  # byte-balanced (unequal counts), then an even split
        types, blob, base, lens = synth.make_batch_host("cfg3b", n, seed=42)
        A = len(types)
        sizes = torch.from_numpy(lens.reshape(n, A).astype(np.int64).sum(axis=1))
        ranges = hdist.shard_ranges(n, world, sizes if n == 301 else None)
        counts = [c for _, c in ranges]
        first, cnt = ranges[rank]

        def oracle_into(t, b, o, l, coords):  # stands in for the gfx950 kernel
            got, err = oracle.hash_batch(t, b, o.numpy().view(np.uint64), l.numpy().view(np.uint32))
            assert err == 0
            coords.copy_(torch.from_numpy(got.view(np.int64)))

        out = torch.full((n, A), -1, dtype=torch.int64)
        mine = hdist.rank_rows(out, counts, rank)
        with _Count() as c:
                full = hdist.hash_sharded(types, blob, torch.from_numpy(base[first:first + cnt].view(np.int64)),
                                      torch.from_numpy(lens[first * A:(first + cnt) * A].view(np.int32)),
                                      counts, out=out, hash_fn=oracle_into)
        ok &= c.n == 1
        want, _ = oracle.hash_batch(types, blob, base, lens)
        ok &= full.data_ptr() == out.data_ptr() == mine.data_ptr() - first * A * 8  # in place
        ok &= bool(np.array_equal(full.numpy().view(np.uint64), want))
        # a separately hashed block is copied into place, then gathered
        again = hdist.allgather_coords(mine.clone(), counts)
        ok &= bool(np.array_equal(again.numpy().view(np.uint64), want))
    ret[rank] = ok
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allgather_matches_single_process(world):
    ctx = mp.get_context("spawn")
    ret = ctx.Manager().dict()
    mp.start_processes(_worker, args=(world, _free_port(), ret), nprocs=world, start_method="spawn")
    assert all(ret[r] for r in range(world))


_EXCHANGE_CASES = ([6, 6, 6], [5, 0, 7], [0, 0, 9], [1, 2, 3], [0, 0, 0])


def _exchange_worker(rank, world, port, want, ret):
    """allgather_coords on rank `rank`'s rows of the mix64 pattern, for each
    case of _EXCHANGE_CASES; the result must equal every device matrix of the
    C++ exchange plan (want[case] = world x N x ROW)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok = True
    for counts, plan_mats in zip(_EXCHANGE_CASES, want):
        N = sum(counts)
        first = sum(counts[:rank])
        e = np.arange(first * 3, (first + counts[rank]) * 3, dtype=np.uint64) + np.uint64(1)
        local = torch.from_numpy(synth.mix64(e).view(np.int64).reshape(counts[rank], 3))
        got = hdist.allgather_coords(local, counts).numpy().view(np.uint64)  # padded form when unequal
        ok &= got.shape == (N, 3)
        for k in range(world):
            ok &= bool(np.array_equal(got.reshape(-1), plan_mats[k]))
    ret[rank] = ok
    dist.destroy_process_group()


def test_exchange_plan_matches_python_gather(tmp_path):
    """The C-ABI device set's exchange plan (hdx_exchange.h, equal / unequal /
    empty shards) leaves every device with the matrix dist.allgather_coords
    gathers on the same shards (world 3, gloo)."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "exchange_dump")
    subprocess.run(["g++", "-std=c++17", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I", os.path.join(root, "hyperdex_amd", "csrc"),
                    os.path.join(root, "tests", "cpp", "exchange_dump.cc"), "-o", exe], check=True)
    world = 3
    want = []
    for i, counts in enumerate(_EXCHANGE_CASES):
        out = str(tmp_path / ("plan%d.bin" % i))
        subprocess.run([exe, out, "3"] + [str(c) for c in counts], check=True)
        mats = np.fromfile(out, dtype=np.uint64).reshape(world, -1) if sum(counts) else np.zeros((world, 0), np.uint64)
        want.append(mats)
    ctx = mp.get_context("spawn")
    ret = ctx.Manager().dict()
    mp.start_processes(_exchange_worker, args=(world, _free_port(), want, ret), nprocs=world, start_method="spawn")
    assert all(ret[r] for r in range(world))


@pytest.mark.gpu
def test_hash_sharded_rccl_world1():
    """The RCCL branch of allgather_coords / hash_sharded in one process."""
    from hyperdex_amd import hashing
    dev = torch.device("cuda", 0)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        types, blob, base, lens = synth.make_batch_device("cfg3b", 5000, device=dev)
        full = hdist.hash_sharded(types, blob, base, lens, [5000])
        want = hashing.hash_batch(types, blob, base, lens)
        torch.cuda.synchronize()
        assert torch.equal(full, want)
        out = torch.empty((5000, len(types)), dtype=torch.int64, device=dev)
        assert hdist.hash_sharded(types, blob, base, lens, [5000], out=out).data_ptr() == out.data_ptr()
        torch.cuda.synchronize()
        assert torch.equal(out, want)
    finally:
        dist.destroy_process_group()
