"""Interleaved A/B of the fused hash + lookup_region forms (run on the GPU box).

    python scripts/ab_fused.py --configs cfg2,cfg3b --forms 100,101,102 --reps 7

Per config one batch and bench.py's two region tables (key subspace, 64
intervals; a 3-attribute subspace, 4 x 4 x 4 cells).  Every round times, back
to back: the separate path (hash_batch + one lookup_region per table, the
automatic kernels), the automatic fused form, and each fused form (debug
variants 100-111,
hdx_kernels_dbg.hip launch_fused_debug; coordinates not written, as in bench.py's
fused line).  The first round checks every form's region ids against the
separate path's.  One JSON line per (config, form): median / min ms.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="cfg2")
    ap.add_argument("--forms", default="100,101")
    ap.add_argument("--objects", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--launches", type=int, default=5)
    args = ap.parse_args()
    import torch

    import bench
    import hyperdex_amd as hdx
    from hyperdex_amd import _lib, synth
    ctx = _lib.debug_library()
    lib = ctx.__enter__()
    dev = torch.device("cuda", 0)
    forms = [int(v) for v in args.forms.split(",")]
    for cfg in args.configs.split(","):
        if cfg == "cfg5":  # the stored-object sweep: forms 47 (64 objects per wave)
            types, *enc = synth.make_encoded_device("cfg3b", args.objects, device=dev)
            blob = base = lens = None

            def hash_into(coords):
                hdx.hash_encoded(types, *enc, coords=coords)

            def fused():
                return hdx.hash_encoded_regions(types, *enc, tables)
        else:
            types, blob, base, lens = synth.make_batch_device(cfg, args.objects, device=dev)

            def hash_into(coords):
                hdx.hash_batch(types, blob, base, lens, coords=coords)

            def fused():
                return hdx.hash_batch_regions(types, blob, base, lens, tables)
        A = len(types)
        tables = bench.key_subspace_tables(A)
        coords = torch.empty((args.objects, A), dtype=torch.int64, device=dev)
        outs = [torch.empty(args.objects, dtype=torch.int64, device=dev) for _ in tables]

        def separate():
            hash_into(coords)
            for t, o in zip(tables, outs):
                hdx.lookup_region(t, coords, out=o)

        times = {v: [] for v in [-2, -1] + forms}
        for rep in range(args.reps + 1):
            for v in [-2, -1] + forms:
                assert lib.hdxdbg_set_kernel_variant(max(v, -1)) >= -1
                fn = separate if v == -2 else fused
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.launches):
                    r = fn()
                e.record()
                torch.cuda.synchronize()
                if rep == 0:
                    if v != -2 and not all(torch.equal(r[k], outs[k]) for k in range(len(tables))):
                        raise SystemExit("fused form %d: region ids differ on %s" % (v, cfg))
                    continue
                times[v].append(s.elapsed_time(e) / args.launches)
        lib.hdxdbg_set_kernel_variant(-1)
        for v in [-2, -1] + forms:
            t = np.array(times[v])
            print(json.dumps({"config": cfg, "form": {-2: "separate", -1: "fused (automatic)"}.get(v, v), "tables": len(tables),
                              "ms_median": round(float(np.median(t)), 4), "ms_min": round(float(t.min()), 4)}),
                  flush=True)
        for t in tables:
            t.close()
        del blob, base, lens, coords, outs
        if cfg == "cfg5":
            del enc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
