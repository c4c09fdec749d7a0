"""Where the regions entry point's time over hash + lookups goes (run on the
GPU box): hdx_hash_batch_regions_device on config 3b with coordinates
returned (no scratch) and without (pooled scratch), the hash alone, and the
lookups alone, interleaved.
    python scripts/regions_overhead.py [--objects N]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=9)
    a = ap.parse_args()
    import torch

    import bench
    import hyperdex_amd as hdx
    from hyperdex_amd import synth
    dev = torch.device("cuda", 0)
    types, blob, base, lens = synth.make_batch_device("cfg3b", a.objects, device=dev)
    A = len(types)
    tables = bench.key_subspace_tables(A)
    coords = torch.empty((a.objects, A), dtype=torch.int64, device=dev)
    outs = [torch.empty(a.objects, dtype=torch.int64, device=dev) for _ in tables]
    cases = {
        "entry_no_coords": lambda: hdx.hash_batch_regions(types, blob, base, lens, tables),
        "entry_with_coords": lambda: hdx.hash_batch_regions(types, blob, base, lens, tables, coords=coords),
        "hash": lambda: hdx.hash_batch(types, blob, base, lens, coords=coords),
        "lookups": lambda: [hdx.lookup_region(t, coords, out=o) for t, o in zip(tables, outs)],
        "hash_then_lookups": lambda: (hdx.hash_batch(types, blob, base, lens, coords=coords),
                                      [hdx.lookup_region(t, coords, out=o) for t, o in zip(tables, outs)]),
    }
    times = {k: [] for k in cases}
    for rep in range(a.reps + 1):
        for k, f in cases.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            f()
            e.record()
            torch.cuda.synchronize()
            if rep:
                times[k].append(s.elapsed_time(e))
    for k, v in times.items():
        print(json.dumps({"case": k, "objects": a.objects, "ms_median": round(float(np.median(v)), 4),
                          "ms_min": round(float(np.min(v)), 4)}), flush=True)


if __name__ == "__main__":
    main()
