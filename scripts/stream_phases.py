"""Per-phase shader cycles of the streamed kernel (debug variants 226: full,
227: skeleton), workgroup 0 wave 0, summed over its batches (run on the GPU box).
    python scripts/stream_phases.py --configs cfg3b,cfg1"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = ["batches", "issue", "store", "describe", "B1", "positions", "B2", "hash", "vm_wait", "B3"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="cfg3b")
    ap.add_argument("--objects", type=int, default=10_000_000)
    a = ap.parse_args()
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import _lib, synth
    dev = torch.device("cuda", 0)
    for cfg in a.configs.split(","):
        types, blob, base, lens = synth.make_batch_device(cfg, a.objects, device=dev)
        coords = torch.empty((a.objects, len(types)), dtype=torch.int64, device=dev)
        for v in (226, 227):
            with _lib.debug_library(v):
                for _ in range(3):
                    hdx.hash_batch(types, blob, base, lens, coords=coords)
                torch.cuda.synchronize()
                ph = coords.view(-1)[:10].cpu().tolist()
            nb = max(ph[0], 1)
            row = {"config": cfg, "variant": v, "batches": ph[0]}
            row.update({NAMES[i]: round(ph[i] / nb, 1) for i in range(1, 10)})
            row["total_per_batch"] = round(sum(ph[1:]) / nb, 1)
            print(json.dumps(row), flush=True)
        del blob, coords
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
