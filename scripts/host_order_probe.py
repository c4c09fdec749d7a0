"""The host-resident path on ordered, shuffled and multi-caller batches
(bench.time_host_path) alone, for rocprofv3 --kernel-trace --stats of the
gather kernel (hdx_gather.hip).  Run on the GPU box."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
import hyperdex_amd as hdx  # noqa: E402
from hyperdex_amd import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3a"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_000
dev = torch.device("cuda", 0)
types, blob, base, lens = synth.make_batch_device(cfg, n, device=dev)
coords = hdx.hash_batch(types, blob, base, lens)
torch.cuda.synchronize()
print(json.dumps({"config": cfg, **bench.time_host_path(types, blob, base, lens, len(types), coords)}), flush=True)
