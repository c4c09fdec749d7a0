"""Interleaved A/B of the wide sweep's forms (debug library; run on the GPU
box): variant -1 (the product: two launches — a lane per object walking the
prefix chain from global memory, then the hash) vs 304 / 305 / 306 (a wave
per object streaming its value through an LDS ring in 4 / 2 / 8 KiB chunks)
and 307 / 308 (304's debug shapes: no hash / no walk), on a key-column store
of the w200 / w1000 schemas.  Usage: ab_wide_sweep.py [schema] [objects]
[v1+v2+...].  Prints one JSON line per form."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch

import hyperdex_amd as hdx
from hyperdex_amd import _lib, synth

schema = sys.argv[1] if len(sys.argv) > 1 else "w200"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
reps = 5
dev = torch.device("cuda", 0)
ctx = _lib.debug_library()
lib = ctx.__enter__()
types, *enc = synth.make_encoded_device(schema, n, device=dev, layout="keycol")
A = len(types)
payload = int(enc[2].to(torch.int64).sum().item()) + int(enc[5].to(torch.int64).sum().item())
algo = payload + n * 24 + n * A * 8
coords = torch.empty((n, A), dtype=torch.int64, device=dev)
ref = None
VARIANTS = tuple(int(x) for x in sys.argv[3].split("+")) if len(sys.argv) > 3 else (-1, 304, 305, 306, 307, 308)
SHAPES = {307, 308}  # debug shapes: WRONG coordinates, not compared
times = {v: [] for v in VARIANTS}
for rep in range(reps + 1):
    for v in VARIANTS:
        lib.hdxdbg_set_kernel_variant(v)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        hdx.hash_encoded(types, *enc, coords=coords)
        e.record()
        torch.cuda.synchronize()
        if rep:
            times[v].append(s.elapsed_time(e))
        if v in SHAPES:
            continue
        got = coords.cpu()
        if ref is None:
            ref = got
        elif not torch.equal(got, ref):
            raise SystemExit("variant %d differs" % v)
for v, t in times.items():
    ms = float(np.median(t))
    print(json.dumps({"schema": schema, "objects": n, "variant": v, "ms_median": round(ms, 4),
                      "frac": round(algo / (ms / 1e3) / 1e9 / 8000.0, 4)}))
