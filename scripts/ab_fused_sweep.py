"""Interleaved A/B of the fused sweep (hdx_hash_encoded_regions_device): the
product form vs debug variants (49: the gather sweep's fused form), with the
two subspace tables of bench.py, coordinates not written (run on the GPU box).
    python scripts/ab_fused_sweep.py --objects 50000000 --variants -1,49"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=50_000_000)
    ap.add_argument("--variants", default="-1,49")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", default="", help="a batch config (cfg3b, ...): time hdx_hash_batch_regions_device instead")
    a = ap.parse_args()
    import torch

    import bench
    import hyperdex_amd as hdx
    from hyperdex_amd import _lib, synth
    dev = torch.device("cuda", 0)
    if a.batch:
        types, *enc = synth.make_batch_device(a.batch, a.objects, device=dev)
        run = lambda tables: hdx.hash_batch_regions(types, *enc, tables)  # noqa: E731
    else:
        types, *enc = synth.make_encoded_device("cfg3b", a.objects, device=dev)
        run = lambda tables: hdx.hash_encoded_regions(types, *enc, tables, coords=False)  # noqa: E731
    A = len(types)
    tables = bench.key_subspace_tables(A)
    variants = [int(v) for v in a.variants.split(",")]
    times = {v: [] for v in variants}
    ref = None
    for rep in range(a.reps + 1):
        for v in variants:
            ctx = _lib.debug_library(v) if v >= 0 else None
            if ctx:
                ctx.__enter__()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            ids = run(tables)
            e.record()
            torch.cuda.synchronize()
            if ctx:
                ctx.__exit__(None, None, None)
            if rep == 0:
                if ref is None:
                    ref = ids.clone()
                elif not torch.equal(ref, ids):
                    raise SystemExit("variant %d differs" % v)
                continue
            times[v].append(s.elapsed_time(e))
    for v in variants:
        t = np.array(times[v])
        print(json.dumps({"fused": a.batch or "cfg5 sweep", "variant": v, "objects": a.objects, "ms_median": round(float(np.median(t)), 3),
                          "ms_min": round(float(t.min()), 3)}), flush=True)


if __name__ == "__main__":
    main()
