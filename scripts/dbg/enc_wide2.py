import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np, torch
import hyperdex_amd as hdx
from hyperdex_amd import synth
from oracle import oracle
from test_encoded import _to_dev
dev = torch.device("cuda", 0)
for A, n in ((33, 65), (33, 66), (33, 127), (33, 128), (33, 129), (17, 65), (17, 100), (5, 70), (1, 70)):
    rules = [synth.Rule(9217, synth.UNIFORM, 0, 130)] * A
    types, blob, base, lens = synth.make_batch_host(rules, n, seed=7)
    enc = synth.encode_values_host(types, blob, base, lens)
    want, _, _ = oracle.hash_encoded(types, *enc)
    got = hdx.hash_encoded(types, *_to_dev(torch, dev, enc)).cpu().numpy().view(np.uint64)
    bad = np.argwhere(got != want)
    slots = [(int(o) % 64) * A + int(j) for o, j in bad]
    print("A", A, "n", n, "mismatches", len(bad), bad[:4].tolist(), "wave-slots", slots[:8], flush=True)
