"""Interleaved A/B of 3b kernel variants in bench.py's secondary context: the
config-3a batch (10.9 GB + coordinates) generated and hashed first and kept
resident, then the config-3b batch generated and the variants timed back to
back (run on the GPU box).

    python scripts/ab_after_3a.py --variants 270/279 --reps 9   ("/" or "," between variants)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="270,279")
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--keep-3a", type=int, default=1)
    args = ap.parse_args()
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import _lib, synth
    lib = _lib.debug_library().__enter__()
    dev = torch.device("cuda", 0)
    n = 10_000_000
    keep = []
    if args.keep_3a:
        t3a = synth.make_batch_device("cfg3a", n, device=dev)
        c3a = torch.empty((n, len(t3a[0])), dtype=torch.int64, device=dev)
        assert lib.hdxdbg_set_kernel_variant(-1) >= -1
        t0 = time.time()
        while time.time() - t0 < 1.0:
            hdx.hash_batch(*t3a, coords=c3a)
        torch.cuda.synchronize()
        keep = [t3a, c3a]
    types, blob, base, lens = synth.make_batch_device("cfg3b", n, device=dev)
    coords = torch.empty((n, len(types)), dtype=torch.int64, device=dev)
    variants = [int(v) for v in args.variants.replace("/", ",").split(",")]
    times = {v: [] for v in variants}
    for rep in range(args.reps + 1):
        for v in variants:
            assert lib.hdxdbg_set_kernel_variant(v) >= -1
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.launches):
                hdx.hash_batch(types, blob, base, lens, coords=coords)
            e.record()
            torch.cuda.synchronize()
            if rep:
                times[v].append(s.elapsed_time(e) / args.launches)
    algo = blob.numel() + n * len(types) * 12
    for v in variants:
        t = np.array(times[v])
        print(json.dumps({"config": "cfg3b", "context": "after 3a (resident)" if args.keep_3a else "alone",
                          "variant": v, "ms_median": round(float(np.median(t)), 4), "ms_min": round(float(t.min()), 4),
                          "frac": round(algo / (np.median(t) / 1e3) / 8e12, 4)}), flush=True)
    del keep


if __name__ == "__main__":
    main()
