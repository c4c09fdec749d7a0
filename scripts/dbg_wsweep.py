"""Debug: where the wave-staged sweep (debug variant) differs from the oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    import torch

    import hyperdex_amd as hdx
    from hyperdex_amd import _lib, synth
    from oracle import oracle
    from test_encoded import _corrupt, _to_dev
    dev = torch.device("cuda", 0)
    v = int(sys.argv[1]) if len(sys.argv) > 1 else 230
    with _lib.debug_library(v):
        for corrupt in (False, True):
            for cfg, n in (("cfg3b", 1001), ("cfg2", 997), ("cfg3b", 16)):
                types, blob, base, lens = synth.make_batch_host(cfg, n, seed=n * 7 + 1)
                enc = synth.encode_values_host(types, blob, base, lens, first_version=5)
                cases = {}
                if corrupt:
                    enc, cases = _corrupt(enc, np.random.default_rng(v + 10))
                want, wver, _ = oracle.hash_encoded(types, *enc)
                versions = torch.zeros(n, dtype=torch.int64, device=dev)
                got = hdx.hash_encoded(types, *_to_dev(torch, dev, enc), versions=versions).cpu().numpy().view(np.uint64)
                gv = versions.cpu().numpy().view(np.uint64)
                bad = np.argwhere(got != want)
                objs = sorted(set(int(i) for i in bad[:, 0])) if bad.size else []
                print(cfg, n, "corrupt" if corrupt else "clean", "mismatches", len(bad), "objects", objs[:20],
                      "kinds", [cases.get(o) for o in objs[:20]], "attrs", sorted(set(int(j) for j in bad[:, 1]))[:20] if bad.size else [],
                      "version mismatches", int((gv != wver).sum()))
                if bad.size:
                    i, j = bad[0]
                    print("  first", i, j, hex(int(got[i, j])), hex(int(want[i, j])), "row got/want zero:", (got[i] == 0).all(), (want[i] == 0).all())


if __name__ == "__main__":
    main()
