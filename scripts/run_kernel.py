"""Run the hash kernel a few times on one synthetic config (profiling target).

    python scripts/run_kernel.py --config cfg3b --variant 12 --launches 3 [--objects N]

Stored-object sweeps: cfg5 / cfg5r / cfg5k (config-3b objects in the columns /
records / key-column layout); cfg5k_w200 / cfg5k_w1000 the wide schemas in a
key column (200 k / 40 k objects unless --objects says otherwise).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3a")
    ap.add_argument("--variant", type=int, default=-1)
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--objects", type=int, default=0)
    a = ap.parse_args()
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import _lib, synth
    ctx = None
    if a.variant >= 0:  # a selected variant runs from the debug library (keep ctx alive:
        ctx = _lib.debug_library(a.variant)  # a collected context manager restores the product lib)
        ctx.__enter__()
    dev = torch.device("cuda", 0)
    cfg, _, schema = a.config.partition("_")
    if not a.objects:
        a.objects = {"w200": 200_000, "w1000": 40_000}.get(schema, 10_000_000)
    if cfg in ("cfg5", "cfg5r", "cfg5k"):  # stored-object sweep over config-3b (or wide) objects
        types, *enc = synth.make_encoded_device(schema or "cfg3b", a.objects, device=dev,
                                                layout={"cfg5r": "records", "cfg5k": "keycol"}.get(cfg, "columns"))
        coords = torch.empty((a.objects, len(types)), dtype=torch.int64, device=dev)
        for _ in range(a.launches):
            hdx.hash_encoded(types, *enc, coords=coords)
    else:
        types, blob, base, lens = synth.make_batch_device(a.config, a.objects, device=dev)
        coords = torch.empty((a.objects, len(types)), dtype=torch.int64, device=dev)
        for _ in range(a.launches):
            hdx.hash_batch(types, blob, base, lens, coords=coords)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
