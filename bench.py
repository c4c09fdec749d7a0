"""bench.py — hyperspace attribute hashing throughput on MI355X.

Metric (BASELINE.json): hashed GiB/s (device-resident) + Mobjects/s on
16-attr x 64 B batches.  Workload at N=1: config 3a of SURVEY §8d —
10M objects, key STRING 64 B + 16 STRING x 64 B (17 coordinates/object),
synthetic bytes generated in HBM.  A step = one launch hashing the whole
batch (every attribute of every object -> coords[n, 17]).

Multi-GPU (torchrun, one rank per GPU): each rank owns its own 10M-object
shard (weak scaling, no collective in the timed region); the RCCL all-gather
of the coordinates is timed separately and reported as `allgather`.

Config 4 rides along in every line as `config4`: one batch
of 100M config-3b objects split over the N ranks by payload bytes
(hyperdex_amd.dist.shard_ranges), each rank hashing its shard straight into
its rows of the full coordinate matrix (hash phase, max over ranks), then the
in-place RCCL all-gather of those rows over xGMI (reported apart), so the
1/2/4/8-GPU runs give config 4's strong-scaling curve.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np


def log(*a):
    print(*a, file=sys.stderr, flush=True)


ROOT = os.path.dirname(os.path.abspath(__file__))
ALGO_EXTRA_PER_ATTR = 4 + 8  # u32 length read + u64 coordinate write
HBM_PEAK_GBPS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg3a")
    ap.add_argument("--objects", type=int, default=0,
                    help="objects per GPU (default 10M; 50M for cfg5, BASELINE config 5)")
    ap.add_argument("--config4-objects", type=int, default=100_000_000,
                    help="config 4: objects of the whole sharded batch (0 = skip)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-allgather", action="store_true")
    ap.add_argument("--no-regions", action="store_true",
                    help="skip the coordinates -> region ids step (SURVEY §8f-1)")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip timing the host-resident (PCIe-inclusive) path")
    ap.add_argument("--no-stream-probe", action="store_true",
                    help="skip the plain streaming-read probe (practical HBM ceiling)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip timing config 3b (16 mixed attrs) beside the config-3a line")
    ap.add_argument("--traffic", default=latest_traffic_file(),
                    help="HBM bytes/launch measured by scripts/gpu_profile.sh (rocprofv3 PMC)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import hyperdex_amd as hdx
    from hyperdex_amd import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # HDX_BENCH_BACKEND=gloo rehearses the multi-rank flow with every rank on
    # cuda:0 (one-GPU box); the real multi-GPU run is one rank per GPU on RCCL.
    backend = os.environ.get("HDX_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    def max_over_ranks(*xs):
        if world == 1:
            return xs
        t = torch.tensor(xs, dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return tuple(float(v) for v in t.tolist())

    cfg, n = args.config, args.objects or (50_000_000 if args.config == "cfg5" else 10_000_000)
    stream = torch.cuda.current_stream(dev)
    if cfg == "cfg5":
        # config 5: reindex sweep over stored objects (values in the daemon's
        # on-disk encoding, keys apart) of the config-3b shape
        types, keys, key_off, key_len, vals, val_off, val_len = synth.make_encoded_device(
            "cfg3b", n, first=rank * n, device=dev)
        A = len(types)
        key_bytes = int(key_len.to(torch.int64).sum().item())
        payload = key_bytes + int(val_len.to(torch.int64).sum().item())
        extra_per_obj = 24  # key_off + val_off (u64) + key_len + val_len (u32)

        def launch():
            hdx.hash_encoded(types, keys, key_off, key_len, vals, val_off, val_len, coords=coords,
                             stream=stream)
    else:
        types, blob, base, lens = synth.make_batch_device(cfg, n, first=rank * n, device=dev)
        A = len(types)
        payload = int(blob.numel())
        extra_per_obj = 8 * 0  # object bases are not counted

        def launch():
            hdx.hash_batch(types, blob, base, lens, coords=coords, stream=stream)
    coords = torch.empty((n, A), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    log("rank %d: %s n=%d A=%d payload %.2f GB" % (rank, cfg, n, A, payload / 1e9))

    # measured ceiling of this access shape beside the spec peak (uses coords
    # as its store target, so it runs before the hash fills them)
    sp = (stream_probe(blob, coords, stream, mix=write_mix(payload, n, A))
          if cfg != "cfg5" and not args.no_stream_probe else None)
    for _ in range(args.warmup):
        launch()
    torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s, e in ev:
        s.record(stream)
        launch()
        e.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    elapsed, kernel_ms = max_over_ranks(elapsed, kernel_ms)

    ms_per_step = elapsed / args.steps * 1e3
    total_payload = payload * world
    total_objs = n * world
    gib_s = total_payload / (ms_per_step / 1e3) / 2**30
    mobj_s = total_objs / (ms_per_step / 1e3) / 1e6
    if cfg == "cfg5":  # value + key bytes, per-object offsets/lengths, coordinates
        algo_bytes = payload + n * extra_per_obj + n * A * 8
    else:  # payload + 4 B length + 8 B coordinate per attribute
        algo_bytes = payload + n * A * ALGO_EXTRA_PER_ATTR
    achieved = algo_bytes / (kernel_ms / 1e3) / 1e9
    traffic, traffic_src = measured_traffic(args.traffic, cfg, n)

    result = {
        "metric": "hashed GiB/s (device-resident) + Mobjects/s, 16-attr×64B batches",
        "value": round(gib_s, 3),
        "unit": "GiB/s",
        "mobjects_per_s": round(mobj_s, 2),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 seed 0x4859504552444558, generated in HBM)",
        "config": {"workload": {"cfg3a": "config 3a", "cfg3b": "config 3b", "cfg2": "config 2",
                                "cfg1": "config 1", "cfg5": "config 5 (reindex sweep, stored 3b objects)"
                                }.get(cfg, cfg) +
                   ": %dM objects/GPU, key + %d attrs" % (n // 1_000_000, A - 1),
                   "objects_per_gpu": n, "attrs": A, "payload_bytes_per_gpu": payload,
                   "parallelism": "shard%d" % world},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel_ms": round(kernel_ms, 4),
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "kernel": hdx.hashing.kernel_for(types, n)[1]},
    }

    if sp is not None:
        result["roofline"]["stream_probe"] = sp
        result["roofline"]["frac_of_probe"] = round(
            achieved / sp.get("read_write_mix_GBps", sp["read_write_1to8_GBps"]), 4)
    if cfg == "cfg5":
        result["roofline"]["kernel"] = ("void hdx::hash_encoded_kernel<false, true, 0, 32, false, false, false>"
                                        "(hdx::EncodedArgs)")
    if world > 1 and not args.no_allgather:
        result["allgather"] = time_allgather(coords, world, dev, backend, max_over_ranks)
        # hash phase then the coordinate exchange, back to back
        result["allgather"]["end_to_end_ms"] = round(kernel_ms + result["allgather"]["ms"], 3)
    if not args.no_regions:
        result["regions"] = time_regions(coords, world, dev, backend, max_over_ranks, stream,
                                         gather=world > 1 and not args.no_allgather)
        if cfg != "cfg5" and A <= 128:
            # ingest's purpose: regions, hashed + looked up in one launch
            result["fused_regions"] = time_fused_batch(
                types, blob, base, lens, n, A, dev, stream, max_over_ranks,
                result["roofline"]["kernel_ms"], result["regions"]["lookup_ms"])
        if cfg == "cfg5":
            # the sweep's purpose: the new regions, decoded + hashed + looked up
            # in one launch with no coordinate written (hdx_hash_encoded_regions_device)
            result["fused_regions"] = time_fused_sweep(
                types, (keys, key_off, key_len, vals, val_off, val_len), n, A, dev, stream, max_over_ranks,
                result["roofline"]["kernel_ms"], result["regions"]["lookup_ms"])

    if not args.no_host_path and rank == 0 and world == 1 and cfg != "cfg5":
        result["host_path"] = time_host_path(types, blob, base, lens, A)

    if rank == 0 and world == 1 and cfg == "cfg3a" and not args.no_secondary:
        # BASELINE's third config with its mixed attribute types, measured the
        # same way in the same run (the headline line stays config 3a's)
        result["secondary"] = {"cfg3b": time_config("cfg3b", n, dev, stream)}

    if args.config4_objects and cfg != "cfg5":
        result["config4"] = time_config4(args.config4_objects, world, rank, dev, stream, max_over_ranks,
                                         backend, gather=not args.no_allgather)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if cfg == "cfg5":
            result["cpu_baseline"] = cpu_baseline_encoded(
                types, (keys, key_off, key_len, vals, val_off, val_len), A, args.cpu_seconds, coords)
        else:
            result["cpu_baseline"] = cpu_baseline(types, blob, base, lens, A, args.cpu_seconds,
                                                  coords)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def time_allgather(coords, world, dev, backend, max_over_ranks, reps=3):
    """RCCL all-gather of every rank's (n, A) u64 coordinates into (world*n, A)
    (hyperdex_amd.dist.allgather_coords), timed apart from the hash phase."""
    import torch
    import torch.distributed as dist

    from hyperdex_amd.dist import allgather_coords
    src = coords if backend == "nccl" else coords[: min(coords.shape[0], 1_000_000)].cpu()
    counts = [src.shape[0]] * world
    out = allgather_coords(src, counts)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = allgather_coords(src, counts)
    torch.cuda.synchronize()
    (dt,) = max_over_ranks((time.perf_counter() - t0) / reps)
    nbytes = out.numel() * 8
    del out
    res = {"ms": round(dt * 1e3, 3), "bytes": nbytes, "backend": backend,
           "busbw_GBps": round(nbytes * (world - 1) / world / dt / 1e9, 2)}
    # the cheaper "gather to host" alternative: every rank
    # copies its own shard to pinned host memory at once
    host = torch.empty(coords.shape, dtype=coords.dtype, pin_memory=True)
    host.copy_(coords, non_blocking=True)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    host.copy_(coords, non_blocking=True)
    torch.cuda.synchronize()
    (d2h,) = max_over_ranks(time.perf_counter() - t0)
    res["d2h_local_shard_ms"] = round(d2h * 1e3, 3)
    res["d2h_GBps_per_gpu"] = round(coords.numel() * 8 / d2h / 1e9, 2)
    del host
    return res


def time_config4(n_total, world, rank, dev, stream, max_over_ranks, backend, gather=True, steps=5):
    """Config 4: one batch of n_total config-3b objects split
    over the ranks by payload bytes.  Every rank derives the same cuts from
    the batch's lengths (dist.shard_ranges on the device), generates its shard
    in HBM, hashes it straight into its rows of the full (n_total, 17)
    coordinate matrix (timed with HIP events, max over ranks = the hash
    phase), then the rows are all-gathered in place (RCCL over xGMI; timed
    apart), and copied to pinned host memory as the cheaper gather-to-host
    alternative.  Strong scaling: the batch is the same at every N."""
    import torch
    import torch.distributed as dist

    from hyperdex_amd import _lib, synth
    from hyperdex_amd import dist as hdist
    from hyperdex_amd.hashing import hash_batch
    rules = synth.CONFIGS["cfg3b"]
    A = len(rules)
    cr = synth.c_rules(rules)
    lib = _lib.lib()
    # the whole batch's lengths, in chunks (identical on every rank), -> sizes
    sizes = torch.empty(n_total, dtype=torch.int64, device=dev)
    chunk = 8_000_000
    tmp = torch.empty(chunk * A, dtype=torch.int32, device=dev)
    for f in range(0, n_total, chunk):
        c = min(chunk, n_total - f)
        _lib.check(lib.hdx_synth_lengths(cr, A, synth.SEED, f, c, tmp.data_ptr(), stream.cuda_stream))
        sizes[f:f + c] = tmp[:c * A].view(c, A).to(torch.int64).sum(dim=1)
    del tmp
    ranges = hdist.shard_ranges(n_total, world, sizes)
    counts = [c for _, c in ranges]
    first, cnt = ranges[rank]
    shard_bytes = int(sizes[first:first + cnt].sum().item())
    del sizes
    types, blob, base, lens = synth.make_batch_device("cfg3b", cnt, first=first, device=dev)
    out = torch.empty((n_total, A), dtype=torch.int64, device=dev)
    mine = hdist.rank_rows(out, counts, rank)

    def run():
        hash_batch(types, blob, base, lens, coords=mine, stream=stream)
    run()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    if world > 1:
        dist.barrier()
    for s, e in ev:
        s.record(stream)
        run()
        e.record(stream)
    torch.cuda.synchronize()
    (hash_ms,) = max_over_ranks(float(np.mean([s.elapsed_time(e) for s, e in ev])))
    payload_total = float(shard_bytes)
    if world > 1:
        t = torch.tensor([payload_total], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t)
        payload_total = float(t.item())
    algo_rank = shard_bytes + cnt * A * ALGO_EXTRA_PER_ATTR
    res = {"workload": "config 4: %dM config-3b objects sharded over %d GPU(s) by payload bytes"
                       % (n_total // 1_000_000, world),
           "objects": n_total, "objects_per_rank": counts, "hash_ms": round(hash_ms, 4),
           "mobjects_per_s": round(n_total / (hash_ms / 1e3) / 1e6, 1),
           "GiB_s": round(payload_total / (hash_ms / 1e3) / 2**30, 2),
           "rank0_roofline_frac": round(algo_rank / (hash_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
           "scaling": "strong"}
    if gather and world > 1:
        src = mine if backend == "nccl" else mine[: min(cnt, 100_000)].cpu()
        cnts = counts if backend == "nccl" else [min(c, 100_000) for c in counts]
        gout = out if backend == "nccl" else None
        hdist.allgather_coords(src, cnts, out=gout)
        torch.cuda.synchronize()
        dist.barrier()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            hdist.allgather_coords(src, cnts, out=gout)
        torch.cuda.synchronize()
        (dt,) = max_over_ranks((time.perf_counter() - t0) / reps)
        nbytes = int(sum(cnts)) * A * 8
        res["allgather"] = {"ms": round(dt * 1e3, 3), "bytes": nbytes, "backend": backend,
                            "equal_counts": len(set(cnts)) == 1,
                            "algbw_GBps": round(nbytes / dt / 1e9, 2),
                            "busbw_GBps": round(nbytes * (world - 1) / world / dt / 1e9, 2)}
        res["end_to_end_ms"] = round(hash_ms + dt * 1e3, 3)
    # gather to host instead: every rank copies its rows to pinned memory at once
    host = torch.empty(mine.shape, dtype=mine.dtype, pin_memory=True)
    host.copy_(mine, non_blocking=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    host.copy_(mine, non_blocking=True)
    torch.cuda.synchronize()
    (d2h,) = max_over_ranks(time.perf_counter() - t0)
    res["d2h_local_rows_ms"] = round(d2h * 1e3, 3)
    del host, out, mine, blob, base, lens
    torch.cuda.empty_cache()
    return res


def key_subspace_tables(A):
    """Region tables of a space like the reference's default: the key subspace
    (attrs {0}) in 64 equal intervals (admin/partition.cc for 1 attribute, 64
    servers) and a 3-attribute subspace {1, 2, 3} in 4 x 4 x 4 cells
    (partition(3, 64) -> 64 regions)."""
    import numpy as np

    from hyperdex_amd import RegionTable
    i = np.arange(64, dtype=np.uint64)
    lo1 = (i << np.uint64(58)).reshape(64, 1)
    up1 = (lo1 + np.uint64((1 << 58) - 1))
    tables = [RegionTable([0], lo1, up1, i + np.uint64(1))]
    if A >= 4:
        c = np.arange(4, dtype=np.uint64)
        cells = np.array([(x, y, z) for x in c for y in c for z in c], np.uint64)
        lo3 = cells << np.uint64(62)
        up3 = lo3 + np.uint64((1 << 62) - 1)
        tables.append(RegionTable([1, 2, 3], lo3, up3, np.arange(65, 129, dtype=np.uint64)))
    return tables


def time_regions(coords, world, dev, backend, max_over_ranks, stream, gather, reps=10):
    """configuration::lookup_region for every object (hdx_lookup_region_device)
    on the key subspace and a 3-attribute subspace, and — multi-GPU — the
    all-gather of the region ids instead of the coordinates."""
    import torch
    import torch.distributed as dist

    from hyperdex_amd import lookup_region
    n, A = coords.shape
    tables = key_subspace_tables(A)
    outs = [torch.empty(n, dtype=torch.int64, device=dev) for _ in tables]
    res = {"objects": n, "tables": [{"dims": int(len(t.attrs)), "regions": int(len(t.ids))}
                                    for t in tables]}
    for t, o in zip(tables, outs):
        lookup_region(t, coords, out=o, stream=stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    torch.cuda.synchronize()
    for s, e in ev:
        s.record(stream)
        for t, o in zip(tables, outs):
            lookup_region(t, coords, out=o, stream=stream)
        e.record(stream)
    torch.cuda.synchronize()
    (ms,) = max_over_ranks(float(np.mean([s.elapsed_time(e) for s, e in ev])))
    res["lookup_ms"] = round(ms, 4)
    res["lookup_mobjects_per_s"] = round(n * world / (ms / 1e3) / 1e6, 1)
    if gather:
        from hyperdex_amd.dist import allgather_coords
        ids = torch.stack(outs, 1).contiguous()
        src = ids if backend == "nccl" else ids[: min(n, 1_000_000)].cpu()
        counts = [src.shape[0]] * world
        allgather_coords(src, counts)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(3):
            out = allgather_coords(src, counts)
        torch.cuda.synchronize()
        (dt,) = max_over_ranks((time.perf_counter() - t0) / 3)
        res["allgather_ids_ms"] = round(dt * 1e3, 3)
        res["allgather_ids_bytes"] = out.numel() * 8
    for t in tables:
        t.close()
    return res


def stream_probe(blob, sink, stream, mix=1, reps=10):
    """Practical HBM ceiling measured in the same run: a plain
    streaming read of the batch's bytes in the hash kernels' access shape
    (hdxdbg_stream_probe), alone, with one 8-byte store per 64 bytes read (the
    1:8 write mix of 64-byte attributes) and, when the config's own mix
    differs, with `mix` stores per 64 bytes (config 2: 3, ≈ its 40 B written
    per 116 B read)."""
    import torch

    import hyperdex_amd as hdx
    lib = hdx.lib()
    res = {}
    for key, write in (("read_GBps", 0), ("read_write_1to8_GBps", 1),
                       ("read_write_mix_GBps", mix if mix != 1 else None)):
        if write is None:
            continue
        nbytes = (blob.numel() // 4096) * 4096
        nbytes = min(nbytes, sink.numel() * 64 // max(write, 1) // 4096 * 4096)
        res.setdefault("bytes", nbytes)

        def go():
            rc = lib.hdxdbg_stream_probe(blob.data_ptr(), nbytes, sink.data_ptr(), write, stream.cuda_stream)
            assert rc == 0, rc
        go()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record(stream)
        for _ in range(reps):
            go()
        e.record(stream)
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / reps
        res[key] = round(nbytes * (1 + write / 8) / (ms / 1e3) / 1e9, 1)
    if mix != 1:
        res["mix_stores_per_64B"] = mix
    return res


def write_mix(payload, n, A):
    """8-byte coordinate stores per 64 bytes read for a packed batch (1..4)."""
    reads = payload + 4 * n * A
    return max(1, min(4, round(64 * (8 * n * A) / reads / 8))) if reads else 1


def time_config(cfg, n, dev, stream, steps=10, warmup=2):
    """Device-resident throughput of another config at the same object count:
    HIP events around each launch on the launch stream, as for the main line."""
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import synth
    types, blob, base, lens = synth.make_batch_device(cfg, n, device=dev)
    A = len(types)
    coords = torch.empty((n, A), dtype=torch.int64, device=dev)
    for _ in range(warmup):
        hdx.hash_batch(types, blob, base, lens, coords=coords, stream=stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    for s, e in ev:
        s.record(stream)
        hdx.hash_batch(types, blob, base, lens, coords=coords, stream=stream)
        e.record(stream)
    torch.cuda.synchronize()
    ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    payload = int(blob.numel())
    algo = payload + n * A * ALGO_EXTRA_PER_ATTR
    res = {"workload": "%s: %dM objects, key + %d attrs" % (cfg, n // 1_000_000, A - 1),
           "GiB_s": round(payload / (ms / 1e3) / 2**30, 3), "mobjects_per_s": round(n / (ms / 1e3) / 1e6, 2),
           "kernel_ms": round(ms, 4), "roofline_frac": round(algo / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
           "kernel": hdx.hashing.kernel_for(types, n)[1]}
    del blob, base, lens, coords
    torch.cuda.empty_cache()
    return res


def time_fused_sweep(types, enc, n, A, dev, stream, max_over_ranks, sweep_ms, lookup_ms, reps=10):
    """hdx_hash_encoded_regions_device over the same stored objects and the
    same two tables as time_regions, coordinates not written; next to the
    sweep + separate lookups it replaces."""
    import torch

    import hyperdex_amd as hdx
    tables = key_subspace_tables(A)
    hdx.hash_encoded_regions(types, *enc, tables, stream=stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    torch.cuda.synchronize()
    for s, e in ev:
        s.record(stream)
        hdx.hash_encoded_regions(types, *enc, tables, stream=stream)
        e.record(stream)
    torch.cuda.synchronize()
    (ms,) = max_over_ranks(float(np.mean([s.elapsed_time(e) for s, e in ev])))
    for t in tables:
        t.close()
    return {"tables": len(tables), "fused_ms": round(ms, 4),
            "separate_ms": round(sweep_ms + lookup_ms, 4),
            "mobjects_per_s": round(n / (ms / 1e3) / 1e6, 2)}


def time_fused_batch(types, blob, base, lens, n, A, dev, stream, max_over_ranks, hash_ms, lookup_ms, reps=10):
    """hdx_hash_batch_regions_device over the same batch and the same two
    tables as time_regions, coordinates not written (the ingest path needs
    only the regions); next to the hash + separate lookups it replaces."""
    import torch

    import hyperdex_amd as hdx
    tables = key_subspace_tables(A)
    hdx.hash_batch_regions(types, blob, base, lens, tables, stream=stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    torch.cuda.synchronize()
    for s, e in ev:
        s.record(stream)
        hdx.hash_batch_regions(types, blob, base, lens, tables, stream=stream)
        e.record(stream)
    torch.cuda.synchronize()
    (ms,) = max_over_ranks(float(np.mean([s.elapsed_time(e) for s, e in ev])))
    for t in tables:
        t.close()
    return {"tables": len(tables), "fused_ms": round(ms, 4),
            "separate_ms": round(hash_ms + lookup_ms, 4),
            "mobjects_per_s": round(n / (ms / 1e3) / 1e6, 2)}


def latest_traffic_file():
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")),
                   key=lambda p: int(os.path.basename(os.path.dirname(p))[1:] or 0))
    return files[-1] if files else ""


def source_digest():
    """sha256 over the kernel and C-ABI sources (what the PMC counters measured):
    a traffic.json recorded from other sources is not this build's traffic."""
    import glob
    import hashlib
    h = hashlib.sha256()
    pats = ("hyperdex_amd/csrc/*.hip", "hyperdex_amd/csrc/*.h", "hyperdex_amd/csrc/*.cpp",
            "hyperdex_amd/csrc/Makefile", "include/*.h")
    for f in sorted(p for pat in pats for p in glob.glob(os.path.join(ROOT, pat))):
        h.update(os.path.relpath(f, ROOT).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def measured_traffic(path, cfg, n):
    """HBM bytes per launch for this config from the committed PMC summary
    (scripts/profile_r2.sh -> scripts/traffic_from_pmc.py), scaled to n, or
    (None, why) when the file was measured on other kernel sources."""
    try:
        doc = json.load(open(path))
        rec = doc[cfg]
    except (OSError, KeyError, ValueError):
        return None, "no PMC record for %s" % cfg
    if doc.get("source_digest") != source_digest():
        return None, "%s measured other kernel sources (digest %s, this build %s)" % (
            os.path.relpath(path, ROOT), doc.get("source_digest"), source_digest())
    per_obj = rec["traffic_bytes"] / rec.get("objects", 10_000_000)
    return int(per_obj * n), "%s (rocprofv3 PMC, digest %s)" % (os.path.relpath(path, ROOT), source_digest())


def time_host_path(types, blob, base, lens, A, n_host=2_000_000):
    """PCIe-inclusive rate: pinned host batch -> hdx_hash_batch_host -> pinned coords."""
    import ctypes

    import hyperdex_amd as hdx
    lib = hdx.lib()
    n = min(n_host, base.numel())
    nb = int((base[n - 1] + lens.view(-1, A)[n - 1].to(dtype=base.dtype).sum()).item()) if n else 0
    ptrs = {}
    for name, nbytes in (("blob", nb), ("base", n * 8), ("lens", n * A * 4), ("out", n * A * 8)):
        p = ctypes.c_void_p()
        hdx._lib.check(lib.hdx_alloc_pinned(nbytes, ctypes.byref(p)))
        ptrs[name] = p.value
    for name, src in (("blob", blob[:nb]), ("base", base[:n]), ("lens", lens[:n * A])):
        host = src.cpu().numpy()  # keep the temporary alive across the copy
        ctypes.memmove(ptrs[name], host.ctypes.data, host.nbytes)
        del host
    t = np.array(types, np.uint32)
    hdx._lib.check(lib.hdx_hash_batch_host(t.ctypes.data, A, ptrs["blob"], nb, ptrs["base"],
                                           ptrs["lens"], n, ptrs["out"]))
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        hdx._lib.check(lib.hdx_hash_batch_host(t.ctypes.data, A, ptrs["blob"], nb, ptrs["base"],
                                               ptrs["lens"], n, ptrs["out"]))
    dt = (time.perf_counter() - t0) / reps
    for p in ptrs.values():
        lib.hdx_free_pinned(p)
    return {"objects": n, "ms": round(dt * 1e3, 3), "GiB_s": round(nb / dt / 2**30, 3),
            "mobjects_per_s": round(n / dt / 1e6, 2)}


def cpu_threads():
    """Every core this process may use: the affinity set, capped by the cgroup's
    CPU quota (on the GPU box 256 logical CPUs are visible but cpu.max allows
    16 cores; 256 threads under that quota measured 3x slower than 16)."""
    quota = cgroup_cpu_quota()
    threads = len(os.sched_getaffinity(0))
    if quota:
        threads = max(1, min(threads, int(quota)))
    return threads, quota


def host_info(threads, quota):
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "threads": threads, "cgroup_cpu_quota_cores": quota,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(types, blob, base, lens, A, seconds, coords):
    """The oracle (C restatement of common/hash.cc, -O2) on this host's cores,
    on a bounded sample of the same batch.  Also verifies the sample's GPU
    coordinates against it (a failed check aborts the bench)."""
    from oracle import oracle
    threads, quota = cpu_threads()
    ns = min(200_000, base.numel())
    nb = int((base[ns - 1] + lens.view(-1, A)[ns - 1].to(dtype=base.dtype).sum()).item())
    hb = blob[:nb].cpu().numpy()
    ho = base[:ns].cpu().numpy().view(np.uint64)
    hl = lens[:ns * A].cpu().numpy().view(np.uint32)
    want, err = oracle.hash_batch(types, hb, ho, hl, nthreads=threads)
    got = coords[:ns].cpu().numpy().view(np.uint64)
    if err or not np.array_equal(got, want):
        raise SystemExit("cpu_baseline: GPU coordinates differ from the oracle")

    def rate(nthreads, budget):
        reps, t0 = 0, time.perf_counter()
        while True:
            oracle.hash_batch(types, hb, ho, hl, nthreads=nthreads)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= budget:
                return reps * nb / dt, reps * ns / dt, reps

    multi_b, multi_o, reps = rate(threads, seconds)
    one_b, one_o, _ = rate(1, max(2.0, seconds / 5))
    return {"value": round(multi_b / 2**30, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "mobjects_per_s": round(multi_o / 1e6, 3),
            "single_thread_GiB_s": round(one_b / 2**30, 3),
            "sample": "%d objects (%.0f MB) of the same batch, %d passes, oracle/hdx_oracle.c -O2 "
                      "pthreads; verified equal to the GPU coords" % (ns, nb / 1e6, reps),
            **host_info(threads, quota)}


def cgroup_cpu_quota():
    """CPU cores the cgroup allows (cpu.max quota / period), None if unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline_encoded(types, enc, A, seconds, coords):
    """Config 5 CPU baseline: the oracle's decode_value + hash on the same
    cores as cpu_baseline (one oracle call per thread over its own chunk of a
    20 k-objects-per-thread sample; ctypes drops the GIL for each call)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle
    threads, quota = cpu_threads()
    keys, key_off, key_len, vals, val_off, val_len = enc
    ns = min(20_000 * threads, val_off.numel())
    ko = key_off[:ns].cpu().numpy().view(np.uint64)
    kl = key_len[:ns].cpu().numpy().view(np.uint32)
    vo = val_off[:ns].cpu().numpy().view(np.uint64)
    vl = val_len[:ns].cpu().numpy().view(np.uint32)
    kend = int((ko.astype(np.uint64) + kl).max())
    vend = int((vo.astype(np.uint64) + vl).max())
    hk, hv = keys[:kend].cpu().numpy(), vals[:vend].cpu().numpy()
    cuts = np.linspace(0, ns, threads + 1).astype(np.int64)
    chunks = [(ko[c0:c1], kl[c0:c1], vo[c0:c1], vl[c0:c1]) for c0, c1 in zip(cuts[:-1], cuts[1:]) if c1 > c0]

    def one(ch):
        return oracle.hash_encoded(types, hk, ch[0], ch[1], hv, ch[2], ch[3])

    with ThreadPoolExecutor(len(chunks)) as pool:
        parts = list(pool.map(one, chunks))
        want = np.concatenate([p[0] for p in parts])
        bad = np.concatenate([p[2] for p in parts])
        if bad.any() or not np.array_equal(coords[:ns].cpu().numpy().view(np.uint64), want):
            raise SystemExit("cpu_baseline: GPU coordinates differ from the oracle")
        nbytes = int(kl.sum()) + int(vl.sum())
        reps, t0 = 0, time.perf_counter()
        while True:
            list(pool.map(one, chunks))
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= seconds:
                break
    return {"value": round(reps * nbytes / dt / 2**30, 3), "unit": "GiB/s", "cores": len(chunks),
            "kind": "port", "mobjects_per_s": round(reps * ns / dt / 1e6, 3),
            "sample": "%d stored objects (%.0f MB), %d passes, oracle hdxo_hash_encoded -O2, %d threads; "
                      "verified equal to the GPU coords" % (ns, nbytes / 1e6, reps, len(chunks)),
            **host_info(len(chunks), quota)}


if __name__ == "__main__":
    main()
