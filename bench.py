"""bench.py — hyperspace attribute hashing throughput on MI355X.

Metric (BASELINE.json): hashed GiB/s (device-resident) + Mobjects/s on
16-attr x 64 B batches.  Workload at N=1: config 3a of SURVEY §8d —
10M objects, key STRING 64 B + 16 STRING x 64 B (17 coordinates/object),
synthetic bytes generated in HBM.  A step = one launch hashing the whole
batch (every attribute of every object -> coords[n, 17]).

Multi-GPU (`--gpus N`, one rank per GPU on RCCL): launched bare, the parent
starts N fresh rank processes itself (before it touches the GPU) and relays
rank 0's line; under torchrun/torch.distributed.run (WORLD_SIZE set) each
process is one rank and WORLD_SIZE must equal --gpus.  Each rank owns its own
10M-object shard (weak scaling, no collective in the timed region); the RCCL
all-gather of the coordinates is timed separately and reported as `allgather`.

Config 4 rides along in every line as `config4`: one batch
of 100M config-3b objects split over the N ranks (hyperdex_amd.dist.
shard_ranges: equal object counts when that keeps every rank within 0.1 % of
its byte share, else byte-balanced cuts), each rank hashing its shard
straight into its rows of the full coordinate matrix (hash phase, max over
ranks), then ONE all-gather of those rows over xGMI (in place for equal
counts, padded otherwise; reported apart), so the 1/2/4/8-GPU runs give
config 4's strong-scaling curve.

HDX_BENCH_DEVICE=cpu (+ HDX_BENCH_BACKEND=gloo) is a CPU rehearsal of the
multi-rank plumbing only — launch, shard cuts, the config-4 gather and the
JSON relay — with a stand-in that writes each object's index instead of its
coordinates (no hashing, no throughput; `value` is null).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np


SWEEP_NUM2 = True  # the product sweep's NUM2 form (config 3b's schema) (hdx_wsweep.hip launch_hash_wsweep_product)


def sweep_kernel_name(layout):
    """The product sweep's kernel (hdx_wsweep.hip launch_hash_wsweep_product) as
    rocprofv3 names it: the record instantiation when keys and values are one
    store (layout "records"), else the other one."""
    return ("void hdx::hash_sweep_wstage_kernel<2, 9728u, 7u, false, true, 0, 14, false, true, true, %s, true, "
            "false, 1, true, 4, %s>(hdx::EncodedArgs)" % ("true" if layout == "records" else "false",
                                                          "true" if SWEEP_NUM2 else "false"))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


ROOT = os.path.dirname(os.path.abspath(__file__))
ALGO_EXTRA_PER_ATTR = 4 + 8  # u32 length read + u64 coordinate write
HBM_PEAK_GBPS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)


CONFIG4_EQUAL_COUNT_TOL = 1e-3  # see shard_ranges(equal_count_tol)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (GPUs); default WORLD_SIZE under a launcher, else 1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--warmup-ms", type=float, default=150.0,
                    help="after the --warmup launches, keep launching untimed until this much "
                         "back-to-back device time has passed (the device's clocks settle over "
                         "the first ~15-40 ms of sustained load, profiles/r3/drift_cfg2.jsonl)")
    ap.add_argument("--config", default="cfg3a")
    ap.add_argument("--objects", type=int, default=0,
                    help="objects per GPU (default 10M; 50M for cfg5, BASELINE config 5)")
    ap.add_argument("--store-layout", default="columns", choices=("columns", "keycol", "records"),
                    help="cfg5's stored objects: 'columns' (each key in place in its packed object, values "
                         "back to back: round 3's layout), 'keycol' (a key column and a value column, "
                         "SURVEY §8d) or 'records' ([key][value] back to back, a LevelDB block's adjacency)")
    ap.add_argument("--store-schema", default="cfg3b",
                    help="cfg5's schema (synth.CONFIGS name; w200 / w1000 for the wide sweep)")
    ap.add_argument("--config4-objects", type=int, default=100_000_000,
                    help="config 4: objects of the whole sharded batch (0 = skip)")
    ap.add_argument("--cfg5-objects", type=int, default=50_000_000,
                    help="config 5 (reindex sweep, key column) in the config-3a line's `secondary` "
                         "(0 = skip)")
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
    return ap.parse_args(argv)


def main():
    args = parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if (args.gpus or 1) > 1:
            # bare `bench.py --gpus N`: start the N ranks here, before anything
            # in this process initialises HIP
            sys.exit(spawn_ranks(args.gpus))
    elif args.gpus is not None and int(env_world) != args.gpus:
        raise SystemExit("bench.py: WORLD_SIZE=%s but --gpus %d" % (env_world, args.gpus))
    if os.environ.get("HDX_BENCH_DEVICE", "cuda") == "cpu":
        return rehearse_cpu(args)
    return run_rank(args)


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(world, grace_s=30.0):
    """Run this script as `world` child processes (RANK = LOCAL_RANK = k,
    WORLD_SIZE, MASTER_ADDR 127.0.0.1, a free MASTER_PORT), relay rank 0's
    stdout (the JSON line) and return non-zero if any rank failed.  When one
    rank fails the others get `grace_s` to exit (they may be blocked in a
    collective) and are then killed by PID."""
    import subprocess
    import tempfile
    port = free_port()
    out0 = tempfile.TemporaryFile()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=out0 if r == 0 else sys.stderr))
    failed_at = None
    while any(p.poll() is None for p in procs):
        if failed_at is None and any(p.returncode not in (None, 0) for p in procs):
            failed_at = time.monotonic()
            log("bench.py: a rank failed (exit codes %s); stopping the others"
                % [p.returncode for p in procs])
        if failed_at is not None and time.monotonic() - failed_at > grace_s:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(0.2)
    codes = [p.wait() for p in procs]
    out0.seek(0)
    for line in out0.read().decode(errors="replace").splitlines():
        # rank 0's JSON line to stdout; anything else it printed (gloo's
        # connection banner) to stderr
        print(line, file=sys.stdout if line.startswith("{") else sys.stderr, flush=True)
    if any(codes):
        log("bench.py: rank exit codes %s" % codes)
        return 1
    return 0


def run_rank(args):
    import torch
    import torch.distributed as dist

    import hyperdex_amd as hdx
    from hyperdex_amd import synth

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
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
        world = dist.get_world_size()
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
            args.store_schema, n, first=rank * n, device=dev, layout=args.store_layout)
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
    sustained_ms = sustain(launch, stream, args.warmup_ms)

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
    traffic_key = pmc_key(cfg, args.store_layout, args.store_schema)
    traffic, traffic_src = measured_traffic(args.traffic, traffic_key, n)

    result = {
        "metric": "hashed GiB/s (device-resident) + Mobjects/s, 16-attr×64B batches",
        "value": round(gib_s, 3),
        "unit": "GiB/s",
        "mobjects_per_s": round(mobj_s, 2),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_sustained_ms": round(sustained_ms, 1),
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 seed 0x4859504552444558, generated in HBM)",
        "config": {"workload": {"cfg3a": "config 3a", "cfg3b": "config 3b", "cfg2": "config 2",
                                "cfg1": "config 1", "cfg5": "config 5 (reindex sweep, stored %s objects)" % args.store_schema
                                }.get(cfg, cfg) +
                   ": %dM objects/GPU, key + %d attrs" % (n // 1_000_000, A - 1),
                   "objects_per_gpu": n, "attrs": A, "payload_bytes_per_gpu": payload,
                   "parallelism": "shard%d" % world,
                   **({"store_layout": args.store_layout} if cfg == "cfg5" else {})},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel_ms": round(kernel_ms, 4),
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "kernel": hdx.hashing.kernel_for(types, n)[1]},
    }

    valu = measured_valu(args.traffic, traffic_key, n, kernel_ms)
    if valu is not None:
        result["roofline"]["valu"] = valu
    if sp is not None:
        result["roofline"]["stream_probe"] = sp
        result["roofline"]["frac_of_probe"] = round(
            achieved / sp.get("read_write_mix_GBps", sp["read_write_1to8_GBps"]), 4)
    if cfg == "cfg5":
        result["roofline"]["kernel"] = (sweep_kernel_name(args.store_layout) if A <= 128
                                        else "hdx::sweep_wide_walk_kernel + hdx::sweep_wide_hash_kernel (EncodedArgs)")
        result["config"]["store_schema"] = args.store_schema
    if world > 1 and not args.no_allgather:
        result["allgather"] = time_allgather(coords, world, dev, backend, max_over_ranks)
        # hash phase then the coordinate exchange, back to back
        result["allgather"]["end_to_end_ms"] = round(kernel_ms + result["allgather"]["ms"], 3)
    # the other configs first, right after the headline's measurement (each with
    # its own warm-up), before the host-path and region extras load the box
    secondary = {}
    if rank == 0 and world == 1 and cfg == "cfg3a" and not args.no_secondary:
        # BASELINE's third config with its mixed attribute types, measured the
        # same way in the same run (the headline line stays config 3a's)
        guarded(secondary, "cfg3b", lambda: time_config("cfg3b", n, dev, stream))
        # BASELINE config 2 (10 M objects) and the GPU side of config 1 (its
        # reference run is CPU-only; 10 M keys here, as in the PMC evidence)
        guarded(secondary, "cfg2", lambda: time_config("cfg2", n, dev, stream))
        guarded(secondary, "cfg1", lambda: time_config("cfg1", n, dev, stream))
        result["secondary"] = secondary

    if not args.no_regions:
        result["regions"] = time_regions(coords, world, dev, backend, max_over_ranks, stream,
                                         gather=world > 1 and not args.no_allgather)
        if cfg != "cfg5" and A <= 128:
            # ingest's purpose: regions, hashed + looked up in one call
            result["regions_entry_point"] = time_fused_batch(
                types, blob, base, lens, n, A, dev, stream, max_over_ranks,
                result["roofline"]["kernel_ms"], result["regions"]["lookup_ms"])
        if cfg == "cfg5":
            # the sweep's purpose: the new regions, decoded + hashed + looked up
            # in one call with no coordinate returned (hdx_hash_encoded_regions_device)
            result["regions_entry_point"] = time_fused_sweep(
                types, (keys, key_off, key_len, vals, val_off, val_len), n, A, dev, stream, max_over_ranks,
                result["roofline"]["kernel_ms"], result["regions"]["lookup_ms"])

    # One-process extras (world 1): a failure is reported in the line, not fatal
    # to it; the device-set runs (every visible device from one process) also
    # under a watchdog that prints the line measured so far.
    if not args.no_host_path and rank == 0 and world == 1:
        if cfg == "cfg5":
            guarded(result, "host_path", lambda: time_host_sweep(
                types, (keys, key_off, key_len, vals, val_off, val_len), A, args.store_layout, coords),
                watchdog_s=DEVICE_SET_WATCHDOG_S, fatal=True)
        else:
            guarded(result, "host_path", lambda: time_host_path(types, blob, base, lens, A, coords),
                    watchdog_s=DEVICE_SET_WATCHDOG_S, fatal=True)

    if args.config4_objects and cfg != "cfg5":
        result["config4"] = time_config4(args.config4_objects, world, rank, dev, stream, max_over_ranks,
                                         backend, gather=not args.no_allgather)
        if world == 1:
            # the same batch through the C-ABI device set: one process drives
            # every visible device (what a C++ daemon links), RCCL gather in-process
            torch.cuda.empty_cache()
            guarded(result, "config4_device_set",
                    lambda: time_config4_device_set(args.config4_objects, dev, stream),
                    watchdog_s=DEVICE_SET_WATCHDOG_S, fatal=True)

    if rank == 0 and world == 1 and cfg == "cfg3a" and not args.no_secondary and args.cfg5_objects:
        # BASELINE config 5 (the reindex sweep at its 50 M objects), after
        # config 4's buffers are gone: 66 GB beside the headline batch
        torch.cuda.empty_cache()
        guarded(secondary, "cfg5", lambda: time_config5(args.cfg5_objects, dev, stream))
        result["secondary"] = secondary

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if cfg == "cfg5":
            guarded(result, "cpu_baseline", lambda: cpu_baseline_encoded(
                types, (keys, key_off, key_len, vals, val_off, val_len), A, args.cpu_seconds, coords))
        else:
            guarded(result, "cpu_baseline", lambda: cpu_baseline(types, blob, base, lens, A, args.cpu_seconds,
                                                                 coords))
            guarded(result, "cpu_per_object",
                    lambda: cpu_per_object_suite(dev, stream, max(1.5, args.cpu_seconds / 3)))

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if FAILED_EXTRAS:
        log("bench.py: device-set extras failed: %s (reported in the line)" % FAILED_EXTRAS)
        return 1
    return 0


# the device-set extras' watchdog: their first run on a node of distinct
# devices must not cost the line (a hang prints what was measured, then exits)
DEVICE_SET_WATCHDOG_S = 300


WATCHDOG_EXIT = 3     # the process exit status after the watchdog printed the line
FAILED_EXTRAS = []    # keys of fatal extras that failed: main() exits non-zero after the line


def guarded(result, key, fn, watchdog_s=None, fatal=False):
    """result[key] = fn(), or {"error": ...} when fn raises.  With watchdog_s,
    a fn still running after that many seconds has result printed as the
    bench line (result[key] an error) and the process ended with status
    WATCHDOG_EXIT (world 1 only): a process that has touched the GPU and
    hung must not look like a success.  With fatal, a failure is still
    reported in the line, and the process exits non-zero after printing it
    (main() reads FAILED_EXTRAS)."""
    import threading
    lock = threading.Lock()  # the line is written by one thread: the watchdog's, or this one
    state = {"done": False}
    timer = None
    if watchdog_s:
        def fire():
            with lock:
                if state["done"]:  # fn returned as the timer fired: its result stands
                    return
                result[key] = {"error": "no result after %d s (watchdog); the line ends here" % watchdog_s}
                print(json.dumps(result), flush=True)
                sys.stderr.flush()
                os._exit(WATCHDOG_EXIT)
        timer = threading.Timer(watchdog_s, fire)
        timer.daemon = True
        timer.start()
    try:
        value = fn()
    except Exception as e:  # an extra's failure is reported in the line
        value = {"error": "%s: %s" % (type(e).__name__, str(e)[:400])}
    with lock:
        state["done"] = True
        result[key] = value
    if timer is not None:
        timer.cancel()
    if fatal and isinstance(value, dict) and "error" in value:
        FAILED_EXTRAS.append(key)


def time_allgather(coords, world, dev, backend, max_over_ranks, reps=3):
    """The all-gather of every rank's (n, A) u64 coordinates into (world*n, A)
    (hyperdex_amd.dist.allgather_coords: one collective), timed apart from the
    hash phase, and the per-rank D2H of the local shard beside it."""
    import torch
    import torch.distributed as dist

    counts = [coords.shape[0]] * world
    if backend == "nccl":
        src = coords
    else:
        counts = rehearsal_counts(counts, rows=1_000_000)
        src = coords[:counts[0]].cpu()
    res, out = time_gather(src, counts, coords.shape[1], None, max_over_ranks, backend, reps)
    del out
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


def time_config4_device_set(n_total, dev0, stream, steps=3):
    """Config 4 through the C-ABI device set (hdx_init_mask over every visible
    device, hdx_hash_batch_device_multi): the batch cut as time_config4 cuts
    it, shard k generated on device 0 and moved to device k, then the hash
    phase (gather = 0) and hash + the in-process RCCL gather (gather = 1),
    each a synchronous call timed on the host clock.  On a one-GPU box the set
    is {0} and the gather a communicator of one."""
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import _lib, synth
    from hyperdex_amd import dist as hdist
    lib = _lib.lib()
    ndev = max(1, lib.hdx_device_count())
    rules = synth.CONFIGS["cfg3b"]
    A = len(rules)
    cr = synth.c_rules(rules)
    sizes = torch.empty(n_total, dtype=torch.int64, device=dev0)
    chunk = 8_000_000
    tmp = torch.empty(chunk * A, dtype=torch.int32, device=dev0)
    for f in range(0, n_total, chunk):
        c = min(chunk, n_total - f)
        _lib.check(lib.hdx_synth_lengths(cr, A, synth.SEED, f, c, tmp.data_ptr(), stream.cuda_stream))
        sizes[f:f + c] = tmp[:c * A].view(c, A).to(torch.int64).sum(dim=1)
    del tmp
    ranges = hdist.shard_ranges(n_total, ndev, sizes, equal_count_tol=CONFIG4_EQUAL_COUNT_TOL)
    shard0_bytes = int(sizes[:ranges[0][1]].sum().item())
    del sizes
    shards, full, own = [], [], []
    for k, (f, c) in enumerate(ranges):
        dk = torch.device("cuda", k)
        types, blob, base, lens = synth.make_batch_device("cfg3b", c, first=f, device=dev0)
        if k:
            blob, base, lens = blob.to(dk), base.to(dk), lens.to(dk)
        torch.cuda.synchronize(dev0)
        shards.append((blob, base, lens))
        full.append(torch.empty((n_total, A), dtype=torch.int64, device=dk))
        own.append(full[-1][:c])  # gather = 0: each shard's own rows
    hdx.init_mask((1 << ndev) - 1)
    try:
        def timed(gather, outs):
            hdx.hash_batch_device_multi(types, shards, gather=gather, coords=outs)  # warm-up
            t0 = time.perf_counter()
            for _ in range(steps):
                hdx.hash_batch_device_multi(types, shards, gather=gather, coords=outs)
            return (time.perf_counter() - t0) / steps * 1e3
        hash_ms = timed(False, own)
        # the exchange's check: sampled rows of every shard as its own device
        # hashed them, then found at the shard's place in every device's matrix
        samples = []
        for k, (f, c) in enumerate(ranges):
            idx = torch.arange(0, c, max(1, c // 4099), device=own[k].device)
            samples.append((f, idx.to(dev0), own[k][idx].to(dev0)))
        both_ms = timed(True, full)
        exchange_ok = all(torch.equal(full[k][f + idx.to(full[k].device)].to(dev0), rows)
                          for k in range(ndev) for f, idx, rows in samples)
    finally:
        hdx.shutdown()
    counts = [c for _, c in ranges]
    res = {"workload": "config 4: %dM config-3b objects over the C-ABI device set of %d GPU(s)"
                       % (n_total // 1_000_000, ndev),
           "devices": ndev, "objects_per_device": counts, "hash_ms": round(hash_ms, 3),
           "mobjects_per_s": round(n_total / (hash_ms / 1e3) / 1e6, 1),
           "device0_roofline_frac": round((shard0_bytes + counts[0] * A * ALGO_EXTRA_PER_ATTR) /
                                          (hash_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
           "hash_and_gather_ms": round(both_ms, 3),
           "gather": "in-place ncclAllGather" if len(set(counts)) == 1 else "grouped in-place ncclBroadcast",
           "exchange_verified": exchange_ok,
           "exchange_check": "every shard's rows (about 4 k sampled per shard, as its own device hashed them) "
                             "at the shard's place in every device's matrix after the exchange",
           "timing": "host clock around synchronous hdx_hash_batch_device_multi calls"}
    del shards, full, own
    torch.cuda.empty_cache()
    return res


def time_config4(n_total, world, rank, dev, stream, max_over_ranks, backend, gather=True, steps=5):
    """Config 4: one batch of n_total config-3b objects split
    over the ranks (shard_ranges with CONFIG4_EQUAL_COUNT_TOL).  Every rank
    derives the same cuts from the batch's lengths (computed on the device),
    generates its shard in HBM, hashes it straight into its rows of the full
    (n_total, 17) coordinate matrix (timed with HIP events, max over ranks =
    the hash phase), then ONE all-gather fills the other ranks' rows (RCCL
    over xGMI; timed apart), and the rows are copied to pinned host memory as
    the cheaper gather-to-host alternative.  Strong scaling: the batch is the
    same at every N."""
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
    ranges = hdist.shard_ranges(n_total, world, sizes, equal_count_tol=CONFIG4_EQUAL_COUNT_TOL)
    imbalance = hdist.byte_imbalance(ranges, sizes) if world > 1 else 0.0
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
    res = {"workload": "config 4: %dM config-3b objects sharded over %d GPU(s)"
                       % (n_total // 1_000_000, world),
           "objects": n_total, "objects_per_rank": counts,
           "shard_byte_imbalance": round(imbalance, 6), "hash_ms": round(hash_ms, 4),
           "mobjects_per_s": round(n_total / (hash_ms / 1e3) / 1e6, 1),
           "GiB_s": round(payload_total / (hash_ms / 1e3) / 2**30, 2),
           "rank0_roofline_frac": round(algo_rank / (hash_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
           "scaling": "strong"}
    if gather and world > 1:
        if backend == "nccl":
            src, cnts, gout = mine, counts, out
        else:  # gloo rehearsal on one GPU: host copies, the same counts pattern
            cnts = rehearsal_counts(counts)
            src, gout = mine[:cnts[rank]].cpu(), None
        res["allgather"], _ = time_gather(src, cnts, A, gout, max_over_ranks, backend)
        res["end_to_end_ms"] = round(hash_ms + res["allgather"]["ms"], 3)
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


def rehearsal_counts(counts, rows=100_000):
    """Per-rank row counts clipped for a host-memory rehearsal, keeping their
    differences (so equal stays equal and unequal stays unequal)."""
    cut = max(0, min(counts) - rows)
    return [int(c) - cut for c in counts]


def time_gather(src, counts, A, out, max_over_ranks, backend, reps=3):
    """hyperdex_amd.dist.allgather_coords of every rank's rows, timed (max
    over ranks), with the number of collectives each gather issued."""
    import torch
    import torch.distributed as dist

    from hyperdex_amd import dist as hdist
    issued = count_collectives()
    got = hdist.allgather_coords(src, counts, out=out)
    if src.is_cuda:
        torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        got = hdist.allgather_coords(src, counts, out=out)
    if src.is_cuda:
        torch.cuda.synchronize()
    (dt,) = max_over_ranks((time.perf_counter() - t0) / reps)
    per_gather = issued.stop() / (reps + 1)
    nbytes = int(sum(counts)) * A * 8
    return {"ms": round(dt * 1e3, 3), "bytes": nbytes, "backend": backend,
            "form": hdist.gather_form(counts), "collectives_per_gather": per_gather,
            "equal_counts": len(set(counts)) == 1,
            "algbw_GBps": round(nbytes / dt / 1e9, 2),
            "busbw_GBps": round(nbytes * (len(counts) - 1) / len(counts) / dt / 1e9, 2)}, got


class count_collectives:
    """Counts torch.distributed collective calls until stop() (wraps the
    module functions allgather_coords may reach)."""
    NAMES = ("all_gather_into_tensor", "all_gather", "broadcast", "all_to_all_single",
             "batch_isend_irecv", "send", "recv", "isend", "irecv")

    def __init__(self):
        import torch.distributed as dist
        self.n, self.saved = 0, {}
        for name in self.NAMES:
            fn = getattr(dist, name)
            self.saved[name] = fn

            def wrap(*a, _fn=fn, **k):
                self.n += 1
                return _fn(*a, **k)
            setattr(dist, name, wrap)

    def stop(self):
        import torch.distributed as dist
        for name, fn in self.saved.items():
            setattr(dist, name, fn)
        return self.n


def rehearse_cpu(args):
    """HDX_BENCH_DEVICE=cpu: the multi-rank plumbing on the host (gloo), no
    hashing.  Same shard cuts and the same single-collective gather as
    config 4, on a batch of --config4-objects (default 200k here) whose rows
    are filled with each object's global index by a stand-in, so the gathered
    matrix can be checked row by row."""
    import torch
    import torch.distributed as dist

    from hyperdex_amd import dist as hdist
    from hyperdex_amd import synth
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group(os.environ.get("HDX_BENCH_BACKEND", "gloo"))
        world = dist.get_world_size()
    rank = dist.get_rank() if world > 1 else 0

    def max_over_ranks(*xs):
        if world == 1:
            return xs
        t = torch.tensor(xs, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return tuple(float(v) for v in t.tolist())

    n_total = args.config4_objects if args.config4_objects != 100_000_000 else 200_000
    rules = synth.CONFIGS["cfg3b"]
    A = len(rules)
    sizes = synth.lengths(rules, n_total).reshape(n_total, A).astype(np.int64).sum(axis=1)
    ranges = hdist.shard_ranges(n_total, world, sizes, equal_count_tol=CONFIG4_EQUAL_COUNT_TOL)
    counts = [c for _, c in ranges]
    first, cnt = ranges[rank]
    out = torch.full((n_total, A), -1, dtype=torch.int64)
    mine = hdist.rank_rows(out, counts, rank)
    mine.copy_(torch.arange(first, first + cnt, dtype=torch.int64)[:, None].expand(cnt, A))
    c4 = {"workload": "config 4 plumbing rehearsal: %d config-3b objects over %d rank(s), no hashing"
                      % (n_total, world),
          "objects": n_total, "objects_per_rank": counts,
          "shard_byte_imbalance": round(hdist.byte_imbalance(ranges, sizes), 6)}
    if world > 1 and not args.no_allgather:
        c4["allgather"], got = time_gather(mine, counts, A, out, max_over_ranks, "gloo", reps=1)
        ok = bool(torch.equal(got, torch.arange(n_total, dtype=torch.int64)[:, None].expand(n_total, A)))
        (bad,) = max_over_ranks(0.0 if ok else 1.0)
        c4["allgather"]["verified"] = bad == 0.0
    result = {"metric": "hashed GiB/s (device-resident) + Mobjects/s, 16-attr×64B batches",
              "value": None, "unit": "GiB/s", "n_gpus": world, "dry_run": "cpu plumbing rehearsal",
              "config4": c4}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


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


def sustain(launch, stream, min_ms):
    """Untimed back-to-back launches until min_ms of device time has passed
    (returns it).  After idle time the device needs tens of milliseconds of
    sustained load before its clocks settle: config 2's 0.31-ms launches drift
    to 0.36-0.44 ms and back over the first ~40 launches, with the kernel or
    with an unrelated 512 MiB fill between launches alike
    (scripts/drift_probe.py, profiles/r3/drift_cfg2.jsonl)."""
    import torch
    if min_ms <= 0:
        torch.cuda.synchronize()
        return 0.0
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(stream)
    launch()
    e.record(stream)
    torch.cuda.synchronize()
    one = max(s.elapsed_time(e), 1e-3)
    reps = max(0, int(np.ceil(min_ms / one)) - 1)
    s.record(stream)
    for _ in range(reps):
        launch()
    e.record(stream)
    torch.cuda.synchronize()
    return one + (s.elapsed_time(e) if reps else 0.0)


def time_config(cfg, n, dev, stream, steps=10, warmup=2, warmup_ms=150.0):
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
    sustain(lambda: hdx.hash_batch(types, blob, base, lens, coords=coords, stream=stream), stream, warmup_ms)
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
    traffic, traffic_src = measured_traffic(latest_traffic_file(), cfg, n)
    res["traffic"] = traffic
    res["traffic_source"] = traffic_src
    valu = measured_valu(latest_traffic_file(), cfg, n, ms)
    if valu is not None:
        res["valu"] = valu
    del blob, base, lens, coords
    torch.cuda.empty_cache()
    return res


def time_config5(n, dev, stream, layout="keycol", steps=10, warmup=2, warmup_ms=150.0):
    """BASELINE config 5 beside the headline line: the reindex
    sweep over n stored config-3b objects (the daemon's value encoding, keys in
    a key column: SURVEY §8d's layout), decoded + hashed in HBM by the product
    sweep (hdx_hash_encoded_device), HIP events around each launch.
    Algorithmic bytes per object: key + value bytes, two u64
    offsets + two u32 lengths, 8 B per coordinate."""
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import synth
    types, *enc = synth.make_encoded_device("cfg3b", n, device=dev, layout=layout)
    A = len(types)
    key_len, val_len = enc[2], enc[5]
    payload = int(key_len.to(torch.int64).sum().item()) + int(val_len.to(torch.int64).sum().item())
    coords = torch.empty((n, A), dtype=torch.int64, device=dev)

    def run():
        hdx.hash_encoded(types, *enc, coords=coords, stream=stream)
    for _ in range(warmup):
        run()
    sustain(run, stream, warmup_ms)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    for s, e in ev:
        s.record(stream)
        run()
        e.record(stream)
    torch.cuda.synchronize()
    ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    algo = payload + n * 24 + n * A * 8
    key = "cfg5" + {"keycol": "k", "records": "r"}.get(layout, "")
    traffic, traffic_src = measured_traffic(latest_traffic_file(), key, n)
    res = {"workload": "config 5 (reindex sweep): %dM stored config-3b objects, %s layout" % (n // 1_000_000, layout),
           "objects": n, "store_layout": layout, "payload_bytes": payload,
           "GiB_s": round(payload / (ms / 1e3) / 2**30, 3), "mobjects_per_s": round(n / (ms / 1e3) / 1e6, 2),
           "kernel_ms": round(ms, 4), "algorithmic_bytes_per_launch": algo,
           "roofline_frac": round(algo / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
           "traffic": traffic, "traffic_source": traffic_src,
           "kernel": sweep_kernel_name(layout)}
    valu = measured_valu(latest_traffic_file(), key, n, ms)
    if valu is not None:
        res["valu"] = valu
    del enc, coords
    torch.cuda.empty_cache()
    return res


def time_fused_sweep(types, enc, n, A, dev, stream, max_over_ranks, sweep_ms, lookup_ms, reps=10):
    """hdx_hash_encoded_regions_device over the same stored objects and the
    same two tables as time_regions, coordinates not returned; next to the
    sweep + separate lookups.  `form`: what the library runs at this size
    (one fused launch, or from 2^20 objects the sweep + per-table lookups
    through pooled scratch; include/hdxhash.h)."""
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
    return {"tables": len(tables), "ms": round(ms, 4),
            "form": "sweep + per-table lookups" if n >= (1 << 20) and A <= 128 else "fused launch",
            "separate_ms": round(sweep_ms + lookup_ms, 4),
            "mobjects_per_s": round(n / (ms / 1e3) / 1e6, 2)}


def time_fused_batch(types, blob, base, lens, n, A, dev, stream, max_over_ranks, hash_ms, lookup_ms, reps=10):
    """hdx_hash_batch_regions_device over the same batch and the same two
    tables as time_regions, coordinates not returned (the ingest path needs
    only the regions); next to the hash + separate lookups.  `form`: what the
    library runs (mixed schemas from 2^20 objects: hash + per-table lookups
    through pooled scratch, else one fused launch; include/hdxhash.h)."""
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
    by_lookup = hdx.hashing.kernel_for(types, n)[0] == 212 and n >= (1 << 20)
    return {"tables": len(tables), "ms": round(ms, 4),
            "form": "hash + per-table lookups" if by_lookup else "fused launch",
            "separate_ms": round(hash_ms + lookup_ms, 4),
            "mobjects_per_s": round(n / (ms / 1e3) / 1e6, 2)}


def latest_traffic_file():
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")),
                   key=lambda p: int(os.path.basename(os.path.dirname(p))[1:] or 0))
    return files[-1] if files else ""


def product_sources():
    """The product library's sources: SRCS and HDRS of hyperdex_amd/csrc/Makefile
    (the debug library's extra kernels are not part of what the PMC counters
    measured, so editing them leaves the digest alone)."""
    names = []
    for line in open(os.path.join(ROOT, "hyperdex_amd", "csrc", "Makefile")):
        if line.startswith(("SRCS :=", "HDRS :=")):
            names += line.split(":=", 1)[1].split()
    return sorted(os.path.normpath(os.path.join(ROOT, "hyperdex_amd", "csrc", f)) for f in names)


def source_digest():
    """sha256 over the product's kernel and C-ABI sources (what the PMC counters
    measured): a traffic.json recorded from other sources is not this build's
    traffic."""
    import hashlib
    h = hashlib.sha256()
    for f in product_sources():
        h.update(os.path.relpath(f, ROOT).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def pmc_key(cfg, store_layout="keycol", store_schema="cfg3b"):
    """The PMC summary's record for a bench line: the config, for config 5 with
    its store layout (cfg5 / cfg5k / cfg5r); its config-5 records are config-3b
    objects, so another store schema names a record the summary does not hold."""
    if cfg != "cfg5":
        return cfg
    key = cfg + {"keycol": "k", "records": "r"}.get(store_layout, "")
    return key if store_schema == "cfg3b" else key + "_" + store_schema


def measured_valu(path, cfg, n, kernel_ms):
    """The VALU-issue roofline of the launch from the same
    digest-matched PMC summary as `traffic`.  `valu_frac` is the PMC pass's own
    ratio: SQ_INSTS_VALU x 4 cycles (a wave64 vector instruction's issue cost
    on one SIMD, MI355X_MICROARCH.md constants table) / (1024 SIMDs x the
    pass's busy cycles, GRBM_GUI_ACTIVE / 8 XCDs) -- instructions and cycles
    from one run.  `valu_frac_at_2p4ghz` divides the same instructions (scaled
    to n) by this run's kernel time at the 2.4 GHz peak clock: a lower bound,
    since the clock under this load is lower.  None when the summary has no
    VALU record or measured other sources."""
    try:
        doc = json.load(open(path))
        rec = doc[cfg]
    except (OSError, KeyError, ValueError):
        return None
    if doc.get("source_digest") != source_digest() or "valu_insts" not in rec:
        return None
    scale = n / rec.get("objects", 10_000_000)
    valu = rec["valu_insts"] * scale
    pmc_cycles = 1024 * rec["grbm_gui_active"] / 8
    return {"valu_frac": round(rec["valu_insts"] * 4 / pmc_cycles, 4),
            "valu_frac_at_2p4ghz": round(valu * 4 / (1024 * 2.4e9 * kernel_ms / 1e3), 4),
            "valu_insts_per_launch": int(valu), "salu_insts_per_launch": int(rec["salu_insts"] * scale),
            "valu_per_wave": round(rec["valu_per_wave"], 1), "salu_per_wave": round(rec["salu_per_wave"], 1),
            "pmc_effective_clock_ghz": round(rec["effective_clock_ghz"], 3),
            "convention": "SQ_INSTS_VALU x 4 cycles / (256 CUs x 4 SIMDs x GRBM_GUI_ACTIVE/8) of the PMC pass"}


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


def time_host_path(types, blob, base, lens, A, coords=None, n_host=2_000_000):
    """PCIe-inclusive rate: pinned host batch -> hdx_hash_batch_host -> pinned coords,
    over the device set of every visible device (hdx_init_mask: the library
    splits the batch byte-balanced over the devices, one worker pipeline each;
    n_host objects per device, at most the resident batch).  With `coords`
    (the device-resident run's), the host path's rows are checked equal."""
    import ctypes

    import hyperdex_amd as hdx
    lib = hdx.lib()
    ndev = max(1, lib.hdx_device_count())
    hdx.init_mask((1 << ndev) - 1)
    devices = hdx.device_set()
    n = min(n_host * len(devices), base.numel())
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
    verified = None
    want = None
    if coords is not None and n:
        want = coords[:n].reshape(-1).cpu().numpy().view(np.uint64)
        got = np.ctypeslib.as_array((ctypes.c_uint64 * (n * A)).from_address(ptrs["out"]))
        verified = bool(np.array_equal(got, want))
        del got
    res = {"objects": n, "devices": len(devices), "ms": round(dt * 1e3, 3),
           "GiB_s": round(nb / dt / 2**30, 3), "GiB_s_per_device": round(nb / dt / 2**30 / len(devices), 3),
           "mobjects_per_s": round(n / dt / 1e6, 2),
           "path": "hdx_init_mask(all visible devices) + hdx_hash_batch_host: pinned H2D, kernel, D2H"}
    if verified is not None:
        res["verified_vs_device_coords"] = verified
    try:
        # the same objects at shuffled places: chunks are packed
        # in index order on the device (hdx_gather.hip), not copied as spans
        res["shuffled"] = time_host_shuffled(lib, t, A, blob, base, lens, n, want)
        # 16 concurrent callers (daemon::loop threads, daemon.cc:345-351), each
        # with its own 1/16 of the ordered batch, after hdx_init_mask
        res["callers16"] = time_host_callers(lib, t, A, ptrs, nb, n, 16, want)
    finally:
        for p in ptrs.values():
            lib.hdx_free_pinned(p)
        hdx.shutdown()  # the set's workers and staging; later phases run on the caller's device
    return res


def time_host_shuffled(lib, t, A, blob, base, lens, n, want, reps=3, block=250_000):
    """hdx_hash_batch_host on the first n objects rewritten in a random order
    (back to back, seeded permutation; built on the device, copied to pinned
    memory): every chunk's span is ~16x its payload, so every chunk is packed."""
    import ctypes

    import torch

    import hyperdex_amd as hdx
    dev = blob.device
    sizes = lens[:n * A].view(n, A).to(torch.int64).sum(dim=1)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED)
    perm = torch.randperm(n, generator=g, device=dev)
    s_perm = sizes[perm]
    start_perm = torch.cumsum(s_perm, 0) - s_perm
    new_base = torch.empty(n, dtype=torch.int64, device=dev)
    new_base[perm] = start_perm
    nb = int(s_perm.sum().item())
    sblob = torch.empty(nb, dtype=torch.uint8, device=dev)
    for k0 in range(0, n, block):  # byte gather, a block of objects at a time
        ks = perm[k0:k0 + block]
        sp, st = s_perm[k0:k0 + block], start_perm[k0:k0 + block]
        seg = torch.repeat_interleave(torch.arange(len(ks), device=dev), sp)
        pos = torch.arange(int(st[0].item()), int(st[0].item()) + int(sp.sum().item()), device=dev)
        src = base[ks][seg] + (pos - st[seg])
        sblob[pos] = blob[src]
        del seg, pos, src
    ptrs = {}
    for name, nbytes in (("blob", nb), ("base", n * 8), ("lens", n * A * 4), ("out", n * A * 8)):
        p = ctypes.c_void_p()
        hdx._lib.check(lib.hdx_alloc_pinned(nbytes, ctypes.byref(p)))
        ptrs[name] = p.value
    try:
        for name, src in (("blob", sblob), ("base", new_base), ("lens", lens[:n * A])):
            host = src.cpu().numpy()
            ctypes.memmove(ptrs[name], host.ctypes.data, host.nbytes)
            del host
        del sblob, new_base, perm, s_perm, start_perm
        torch.cuda.empty_cache()
        call = lambda: hdx._lib.check(lib.hdx_hash_batch_host(t.ctypes.data, A, ptrs["blob"], nb, ptrs["base"],
                                                              ptrs["lens"], n, ptrs["out"]))
        call()
        t0 = time.perf_counter()
        for _ in range(reps):
            call()
        dt = (time.perf_counter() - t0) / reps
        res = {"objects": n, "ms": round(dt * 1e3, 3), "GiB_s": round(nb / dt / 2**30, 3),
               "order": "random permutation of the objects, back to back (pinned)",
               "path": "chunks packed in index order by hdx_gather.hip from the pinned batch"}
        if want is not None:
            got = np.ctypeslib.as_array((ctypes.c_uint64 * (n * A)).from_address(ptrs["out"]))
            res["verified_vs_device_coords"] = bool(np.array_equal(got, want))
            del got
        return res
    finally:
        for p in ptrs.values():
            lib.hdx_free_pinned(p)


def time_host_callers(lib, t, A, ptrs, nb, n, callers, want, reps=3):
    """`callers` long-lived threads (as daemon::loop threads are) at once,
    each hdx_hash_batch_host on its own contiguous 1/callers of the pinned
    batch (ctypes releases the GIL in the call): the aggregate rate of a round
    in which every caller makes one call, after one untimed round (each thread
    binds its pipeline on its first call)."""
    import ctypes
    import threading

    cuts = [n * k // callers for k in range(callers + 1)]
    start = threading.Barrier(callers + 1)
    done = threading.Barrier(callers + 1)
    errs = []

    def worker(k):
        f, c = cuts[k], cuts[k + 1] - cuts[k]
        for _ in range(reps + 1):
            start.wait()
            if c:
                st = lib.hdx_hash_batch_host(t.ctypes.data, A, ptrs["blob"], nb, ptrs["base"] + 8 * f,
                                             ptrs["lens"] + 4 * A * f, c, ptrs["out"] + 8 * A * f)
                if st != 0:
                    errs.append((k, st, lib.hdx_last_error()))
            done.wait()

    th = [threading.Thread(target=worker, args=(k,), daemon=True) for k in range(callers)]
    for x in th:
        x.start()
    dts = []
    for r in range(reps + 1):
        t0 = time.perf_counter()
        start.wait()
        done.wait()
        if r:
            dts.append(time.perf_counter() - t0)
    for x in th:
        x.join()
    if errs:
        raise RuntimeError("callers failed: %s" % errs[:3])
    dt = float(np.mean(dts))
    res = {"callers": callers, "objects": n, "ms": round(dt * 1e3, 3), "GiB_s": round(nb / dt / 2**30, 3),
           "threads": "long-lived, one call each per round"}
    if want is not None:
        got = np.ctypeslib.as_array((ctypes.c_uint64 * (n * A)).from_address(ptrs["out"]))
        res["verified_vs_device_coords"] = bool(np.array_equal(got, want))
        del got
    return res


def time_host_sweep(types, enc, A, layout, coords, n_host=1_000_000):
    """Config 5 from host memory (hdx_hash_encoded_host, the indexer's entry
    point): a pinned host copy of the first n_host objects per device of the
    store (keys, values, offsets, lengths), swept over the device set of every
    visible device (cut byte-balanced, one 128 MiB-chunk PCIe pipeline per
    device), coordinates and versions back into pinned host arrays.  The
    host coordinates are checked equal to the device-resident sweep's."""
    import ctypes

    import hyperdex_amd as hdx
    lib = hdx.lib()
    ndev = max(1, lib.hdx_device_count())
    hdx.init_mask((1 << ndev) - 1)
    devices = hdx.device_set()
    keys, key_off, key_len, vals, val_off, val_len = enc
    n = min(n_host * len(devices), val_off.numel())
    ko = key_off[:n].cpu().numpy().view(np.uint64)
    kl = key_len[:n].cpu().numpy().view(np.uint32)
    vo = val_off[:n].cpu().numpy().view(np.uint64)
    vl = val_len[:n].cpu().numpy().view(np.uint32)
    kend = int((ko + kl).max())
    vend = int((vo + vl).max())
    records = layout == "records"
    ptrs = {}
    sizes = {"keys": kend, "vals": 0 if records else vend, "ko": n * 8, "kl": n * 4, "vo": n * 8, "vl": n * 4,
             "out": n * A * 8, "ver": n * 8}
    if records:
        sizes["keys"] = max(kend, vend)
    for name, nbytes in sizes.items():
        if nbytes == 0:
            continue
        p = ctypes.c_void_p()
        hdx._lib.check(lib.hdx_alloc_pinned(nbytes, ctypes.byref(p)))
        ptrs[name] = p.value
    srcs = [("keys", keys[:sizes["keys"]]), ("ko", ko), ("kl", kl), ("vo", vo), ("vl", vl)]
    if not records:
        srcs.append(("vals", vals[:vend]))
    for name, src in srcs:
        host = src.cpu().numpy() if hasattr(src, "cpu") else src
        ctypes.memmove(ptrs[name], host.ctypes.data, host.nbytes)
        del host
    vptr, vbytes = (ptrs["keys"], sizes["keys"]) if records else (ptrs["vals"], vend)
    t = np.array(types, np.uint32)

    def call():
        hdx._lib.check(lib.hdx_hash_encoded_host(t.ctypes.data, A, ptrs["keys"], sizes["keys"], ptrs["ko"], ptrs["kl"],
                                                 vptr, vbytes, ptrs["vo"], ptrs["vl"], n, ptrs["out"], ptrs["ver"]))
    call()
    got = np.ctypeslib.as_array((ctypes.c_uint64 * (n * A)).from_address(ptrs["out"])).reshape(n, A)
    if not np.array_equal(got, coords[:n].cpu().numpy().view(np.uint64)):
        raise SystemExit("host_path: hdx_hash_encoded_host coordinates differ from the device-resident sweep's")
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        call()
    dt = (time.perf_counter() - t0) / reps
    for p in ptrs.values():
        lib.hdx_free_pinned(p)
    hdx.shutdown()
    nb = int(kl.astype(np.uint64).sum()) + int(vl.astype(np.uint64).sum())
    return {"objects": n, "devices": len(devices), "ms": round(dt * 1e3, 3),
            "GiB_s": round(nb / dt / 2**30, 3), "GiB_s_per_device": round(nb / dt / 2**30 / len(devices), 3),
            "mobjects_per_s": round(n / dt / 1e6, 2), "store_layout": layout,
            "path": "hdx_init_mask(all visible devices) + hdx_hash_encoded_host: pinned H2D of key / value spans, "
                    "sweep, D2H of coordinates and versions; equal to the device-resident sweep's coordinates"}


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


CPU_PASSES = 5  # the baseline's passes: a pass disturbed by the box's other tenants stays out of the median


def pinned_passes(work, seconds, passes=CPU_PASSES):
    """Times `work` (one (prepare, run, nbytes, nobj) per thread) on threads
    pinned one per CPU of this process's affinity set.  Each thread first
    touches its own copy of its chunk (prepare(), on that thread: its pages
    land on its NUMA node), then in each of `passes` passes of seconds /
    passes every thread runs its chunk until the pass's deadline.  Returns the
    per-pass (bytes/s, objects/s) list and the median pass.  ctypes drops the
    GIL for each oracle call, so the threads run in parallel."""
    import threading
    cpus = sorted(os.sched_getaffinity(0))
    n = len(work)
    ready = threading.Barrier(n + 1)  # every thread prepared and warm before pass 0's clock starts
    start = threading.Barrier(n + 1)
    done = threading.Barrier(n + 1)
    reps = [[0] * passes for _ in range(n)]
    deadline = [0.0]
    errors = []

    def worker(k):
        try:
            os.sched_setaffinity(0, {cpus[k % len(cpus)]})  # this thread only (Linux: pid 0 = the caller)
        except OSError:
            pass
        try:
            prepare, run, _, _ = work[k]
            state = prepare()
            run(state)  # warm: first-call page faults and allocations stay out of the passes
            ready.wait()
            for p in range(passes):
                start.wait()
                while time.perf_counter() < deadline[0]:
                    run(state)
                    reps[k][p] += 1
                done.wait()
        except threading.BrokenBarrierError:
            pass
        except Exception as e:  # noqa: BLE001 — re-raised on the main thread
            errors.append(e)
            ready.abort()
            start.abort()
            done.abort()
    ths = [threading.Thread(target=worker, args=(k,), daemon=True) for k in range(n)]
    for th in ths:
        th.start()
    rates = []
    try:
        ready.wait()
        for p in range(passes):
            deadline[0] = time.perf_counter() + seconds / passes
            t0 = time.perf_counter()
            start.wait()
            done.wait()
            dt = time.perf_counter() - t0
            nb = sum(reps[k][p] * work[k][2] for k in range(n))
            no = sum(reps[k][p] * work[k][3] for k in range(n))
            rates.append((nb / dt, no / dt))
    except threading.BrokenBarrierError:
        pass
    for th in ths:
        th.join()
    if errors:
        raise errors[0]
    med = sorted(rates)[len(rates) // 2]
    return rates, med, sum(sum(r) for r in reps)


def cpu_baseline(types, blob, base, lens, A, seconds, coords):
    """The oracle (C restatement of common/hash.cc, -O2) on this host's cores,
    on a bounded sample of the same batch: one pinned thread per core, each
    over its own first-touched copy of a contiguous chunk (pinned_passes),
    median of 5 passes.  Also verifies the sample's GPU coordinates against
    it (a failed check aborts the bench)."""
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
    sizes = hl.reshape(ns, A).astype(np.uint64).sum(axis=1)
    cuts = np.linspace(0, ns, threads + 1).astype(np.int64)

    def job(c0, c1):
        lo, hi = int(ho[c0]), int(ho[c1 - 1] + sizes[c1 - 1])

        def prepare():  # this thread's compact copy of its objects
            return (hb[lo:hi].copy(), (ho[c0:c1] - np.uint64(lo)).copy(), hl[c0 * A:c1 * A].copy())

        def run(st):
            oracle.hash_batch(types, st[0], st[1], st[2], nthreads=1)
        return prepare, run, hi - lo, c1 - c0
    work = [job(int(c0), int(c1)) for c0, c1 in zip(cuts[:-1], cuts[1:]) if c1 > c0]
    rates, (mb, mo), reps = pinned_passes(work, seconds)
    one, (ob, _), _ = pinned_passes(work[:1], max(1.5, seconds / 5), passes=1)
    return {"value": round(mb / 2**30, 3), "unit": "GiB/s", "cores": len(work), "kind": "port",
            "mobjects_per_s": round(mo / 1e6, 3),
            "passes_GiB_s": [round(r[0] / 2**30, 3) for r in rates],
            "single_thread_GiB_s": round(ob / 2**30, 3),
            "sample": "%d objects (%.0f MB) of the same batch, oracle/hdx_oracle.c -O2, one pinned thread per core "
                      "over its own first-touched copy of a contiguous chunk, median of 5 passes (%d chunk passes); "
                      "verified equal to the GPU coords" % (ns, nb / 1e6, reps),
            **host_info(len(work), quota)}


def cpu_per_object(types, blob, base, lens, coords, seconds, label):
    """The product's own per-object CPU path (hdx_hash_object / hdx_hash_key,
    what the C++ drop-in include/hyperdex_amd/hash.h runs for
    common/hash.cc:48-68) timed the way daemon threads call it: one
    synchronous call per object (tools/libhdxcpubench.so), single thread and
    over this host's quota of cores, on a sample of the given batch (host
    numpy arrays); its output is checked against `coords` (the GPU's)."""
    import ctypes
    threads, quota = cpu_threads()
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libhdxcpubench.so"))
    fn = lib.hdxcpu_time_objects
    fn.restype = ctypes.c_int
    vp = ctypes.c_void_p
    fn.argtypes = [vp, ctypes.c_uint32, vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_int, ctypes.c_int,
                   ctypes.c_double, vp, vp]
    A = len(types)
    n = len(base)
    t = np.ascontiguousarray(types, np.uint32)
    out = np.zeros((n, A), np.uint64)
    key_only = 1 if A == 1 else 0
    nbytes = int(lens.astype(np.uint64).sum())

    def run(nthreads, budget):
        passes, secs = ctypes.c_uint64(), ctypes.c_double()
        rc = fn(t.ctypes.data, A, blob.ctypes.data, base.ctypes.data, lens.ctypes.data, n, out.ctypes.data,
                nthreads, key_only, budget, ctypes.byref(passes), ctypes.byref(secs))
        if rc != 0:
            raise SystemExit("cpu_per_object: hdx status %d" % rc)
        return passes.value, secs.value

    run(1, 0.0)
    if not np.array_equal(out, coords.reshape(n, A)):
        raise SystemExit("cpu_per_object: %s coordinates differ from the GPU's" % label)
    p1, s1 = run(1, seconds / 3)
    pm, sm = run(threads, seconds * 2 / 3)
    return {"workload": label, "objects": n, "bytes": nbytes,
            "ns_per_object_1thread": round(s1 / (p1 * n) * 1e9, 1),
            "mobjects_per_s_1thread": round(p1 * n / s1 / 1e6, 3),
            "GiB_s_1thread": round(p1 * nbytes / s1 / 2**30, 3),
            "cores": threads, "mobjects_per_s": round(pm * n / sm / 1e6, 3),
            "GiB_s": round(pm * nbytes / sm / 2**30, 3),
            "verified_vs_gpu": True}


def cpu_per_object_suite(dev, stream, seconds):
    """cpu_per_object on config 1 (1 M 64-byte keys, BASELINE's CPU-only
    config) and config 3b (the mixed 16-attribute object); each sample's GPU
    coordinates come from the product kernel on the same bytes."""
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import synth
    threads, quota = cpu_threads()
    res = {"kind": "product per-object CPU path (hdx_hash_object / hdx_hash_key via libhdxcpubench)",
           **host_info(threads, quota), "configs": {}}
    samples = [("config 1: 64-byte key, hash(schema, key, &h)", "cfg1", 1_000_000),
               ("config 3b: key + 16 mixed attrs, hash(schema, key, value, hs)", "cfg3b", 100_000)]
    for label, cfg, n in samples:
        types, blob, base, lens = synth.make_batch_host(cfg, n)
        tb = torch.from_numpy(blob).to(dev)
        to = torch.from_numpy(base.view(np.int64)).to(dev)
        tl = torch.from_numpy(lens.view(np.int32)).to(dev)
        got = hdx.hash_batch(types, tb, to, tl, stream=stream)
        torch.cuda.synchronize()
        gpu = got.cpu().numpy().view(np.uint64)
        res["configs"][cfg] = cpu_per_object(types, blob, base, lens, gpu, seconds, label)
        del tb, to, tl, got
    return res


def cgroup_cpu_quota():
    """CPU cores the cgroup allows (cpu.max quota / period), None if unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def verify_encoded_spread(types, enc, coords, oracle, sample=2048, seed=5):
    """The sweep's coordinates of objects spread over the whole store (the last
    64 and `sample` random ones) against the oracle, each object's key and
    value bytes copied to the host on their own; returns the count checked."""
    keys, key_off, key_len, vals, val_off, val_len = enc
    n = val_off.numel()
    if n == 0:
        return 0
    rng = np.random.default_rng(seed)
    idx = np.unique(np.concatenate([rng.integers(0, n, min(sample, n)), np.arange(max(0, n - 64), n)]))
    it = torch_index(idx, key_off.device)
    ko = key_off[it].cpu().numpy().view(np.uint64)
    kl = key_len[it].cpu().numpy().view(np.uint32)
    vo = val_off[it].cpu().numpy().view(np.uint64)
    vl = val_len[it].cpu().numpy().view(np.uint32)
    kparts, vparts = [], []
    for i in range(len(idx)):
        kparts.append(keys[int(ko[i]):int(ko[i]) + int(kl[i])].cpu().numpy())
        vparts.append(vals[int(vo[i]):int(vo[i]) + int(vl[i])].cpu().numpy())
    nko = np.concatenate([[0], np.cumsum(kl.astype(np.uint64))[:-1]]).astype(np.uint64)
    nvo = np.concatenate([[0], np.cumsum(vl.astype(np.uint64))[:-1]]).astype(np.uint64)
    hk = np.concatenate(kparts) if kparts else np.zeros(0, np.uint8)
    hv = np.concatenate(vparts) if vparts else np.zeros(0, np.uint8)
    want, _, bad = oracle.hash_encoded(types, hk, nko, kl, hv, nvo, vl)
    got = coords[it].cpu().numpy().view(np.uint64)
    if bad.any() or not np.array_equal(got, want):
        raise SystemExit("cpu_baseline: GPU coordinates of objects spread over the store differ from the oracle")
    return len(idx)


def torch_index(idx, device):
    import torch
    return torch.from_numpy(idx.astype(np.int64)).to(device)


def cpu_baseline_encoded(types, enc, A, seconds, coords):
    """Config 5 CPU baseline: the oracle's decode_value + hash, one pinned
    thread per core as cpu_baseline, each over its own first-touched compact
    copy (keys back to back, values back to back) of a 20 k-object chunk, so
    every store layout times the same work; median of 5 passes.  The
    sample's GPU coordinates, and those of objects spread over the whole
    store, are checked against the oracle first."""
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
    want, _, bad = oracle.hash_encoded(types, hk, ko, kl, hv, vo, vl)
    if bad.any() or not np.array_equal(coords[:ns].cpu().numpy().view(np.uint64), want):
        raise SystemExit("cpu_baseline: GPU coordinates differ from the oracle")
    spread = verify_encoded_spread(types, enc, coords, oracle)
    cuts = np.linspace(0, ns, threads + 1).astype(np.int64)

    def compact(buf, off, ln):
        out = np.empty(int(ln.astype(np.uint64).sum()), np.uint8)
        noff = np.zeros(len(off), np.uint64)
        if len(off) > 1:
            noff[1:] = np.cumsum(ln[:-1].astype(np.uint64))
        for i in range(len(off)):
            out[int(noff[i]):int(noff[i]) + int(ln[i])] = buf[int(off[i]):int(off[i]) + int(ln[i])]
        return out, noff

    def job(c0, c1):
        def prepare():  # this thread's compact copy of its objects
            k, nko = compact(hk, ko[c0:c1], kl[c0:c1])
            v, nvo = compact(hv, vo[c0:c1], vl[c0:c1])
            return k, nko, kl[c0:c1].copy(), v, nvo, vl[c0:c1].copy()

        def run(st):
            oracle.hash_encoded(types, *st)
        return prepare, run, int(kl[c0:c1].sum()) + int(vl[c0:c1].sum()), c1 - c0
    work = [job(int(c0), int(c1)) for c0, c1 in zip(cuts[:-1], cuts[1:]) if c1 > c0]
    rates, (mb, mo), reps = pinned_passes(work, seconds)
    nbytes = int(kl.sum()) + int(vl.sum())
    return {"value": round(mb / 2**30, 3), "unit": "GiB/s", "cores": len(work), "kind": "port",
            "mobjects_per_s": round(mo / 1e6, 3),
            "passes_GiB_s": [round(r[0] / 2**30, 3) for r in rates],
            "sample": "%d stored objects (%.0f MB), oracle hdxo_hash_encoded -O2, one pinned thread per core over its "
                      "own first-touched compact copy (keys and values back to back, whatever the store's layout) "
                      "of a contiguous chunk, median of 5 passes (%d chunk passes); verified equal to the GPU coords, "
                      "and %d objects spread over the whole store (the last 64 and random ones)"
                      % (ns, nbytes / 1e6, reps, spread),
            **host_info(len(work), quota)}


if __name__ == "__main__":
    sys.exit(main())
