"""Interleaved in-process A/B of hash kernel variants (run on the GPU box).

    python scripts/ab_variants.py --configs cfg3a,cfg3b --variants 0,7,8 --reps 7 --launches 5

One batch per config is generated in HBM once; then for `reps` rounds every
variant is timed back to back (HIP events around `launches` launches), so the
variants see the same clocks and the same box.  Prints one JSON line per
(config, variant) with the median and min kernel time and the roofline frac.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="cfg3a")
    ap.add_argument("--variants", default="0,7")
    ap.add_argument("--objects", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--check", default="", help="variants whose coordinates must equal the first's "
                    "(default: all but the debug shapes, which write wrong coordinates)")
    args = ap.parse_args()
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import _lib, synth
    ctx = _lib.debug_library()  # the A/B selection lives in libhdxhash_dbg.so only
    lib = ctx.__enter__()
    dev = torch.device("cuda", 0)
    variants = [int(v) for v in args.variants.split(",")]
    checked = set(int(v) for v in args.check.split(",")) if args.check else set(variants) - {40, 41, 57, 58, 207, 208, 218, 241, 297, 313, 314, 315, 223, 224, 225, 226, 227, 237, 238, 248, 249, 252}
    for cfg in args.configs.split(","):
        if cfg in ("cfg5", "cfg5r", "cfg5k"):  # stored-object sweep; cfg5r / cfg5k: records / key column
            types, *enc = synth.make_encoded_device("cfg3b", args.objects, device=dev,
                                                    layout={"cfg5r": "records", "cfg5k": "keycol"}.get(cfg, "columns"))
            blob = enc[0][:int(enc[2].to(torch.int64).sum().item())]  # key bytes ...
            extra = int(enc[5].to(torch.int64).sum().item())            # ... + value bytes

            def run(coords):
                hdx.hash_encoded(types, *enc, coords=coords)
        else:
            types, blob, base, lens = synth.make_batch_device(cfg, args.objects, device=dev)
            extra = 0

            def run(coords):
                hdx.hash_batch(types, blob, base, lens, coords=coords)
        A = len(types)
        coords = torch.empty((args.objects, A), dtype=torch.int64, device=dev)
        ref = None
        times = {v: [] for v in variants}
        for rep in range(args.reps + 1):
            for v in variants:
                assert lib.hdxdbg_set_kernel_variant(v) >= -1
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.launches):
                    run(coords)
                e.record()
                torch.cuda.synchronize()
                if rep == 0:  # warm-up round doubles as a cross-variant equality check
                    if ref is None:
                        ref = coords.clone()
                    elif v in checked and not torch.equal(ref, coords):
                        raise SystemExit("variant %d differs from variant %d on %s" % (v, variants[0], cfg))
                    continue
                times[v].append(s.elapsed_time(e) / args.launches)
        algo = blob.numel() + extra + args.objects * A * 12
        for v in variants:
            t = np.array(times[v])
            print(json.dumps({"config": cfg, "variant": v, "ms_median": round(float(np.median(t)), 4),
                              "ms_min": round(float(t.min()), 4),
                              "frac": round(algo / (np.median(t) / 1e3) / 8e12, 4)}), flush=True)
        del blob, coords, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
