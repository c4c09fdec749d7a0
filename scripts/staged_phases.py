"""Per-phase shader cycles of the LDS-staged sweep (debug variant 71) on
config 5: window store + metadata issue, prefix walk, next span + window
issue, hash passes; averaged over the persistent waves (run on the GPU box)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import synth
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    dev = torch.device("cuda", 0)
    assert hdx.lib().hdxdbg_set_kernel_variant(71) >= -1
    types, *enc = synth.make_encoded_device("cfg3b", n, device=dev)
    blocks = 256 * 64
    versions = torch.zeros(n + 4 * blocks, dtype=torch.int64, device=dev)
    for _ in range(2):
        hdx.hash_encoded(types, *enc, versions=versions)
    torch.cuda.synchronize()
    ph = versions[n:].cpu().numpy().reshape(-1, 4)
    ph = ph[ph.sum(1) > 0]
    groups = (n + 6) // 7
    per = ph.sum(0) / groups * len(ph)  # cycles per group per wave
    names = ["store+meta", "walk", "span+issue", "hash"]
    print({"waves": len(ph), **{k: round(float(v) / len(ph), 1) for k, v in zip(names, per)}})


if __name__ == "__main__":
    main()
