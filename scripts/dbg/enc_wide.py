import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np, torch
import hyperdex_amd as hdx
from hyperdex_amd import synth
from oracle import oracle
from test_encoded import _to_dev
dev = torch.device("cuda", 0)
for A in (33, 64, 65, 70):
    rules = [synth.Rule(9217, synth.UNIFORM, 0, 130)] * A
    types, blob, base, lens = synth.make_batch_host(rules, 130, seed=7)
    enc = synth.encode_values_host(types, blob, base, lens)
    want, _, _ = oracle.hash_encoded(types, *enc)
    got = hdx.hash_encoded(types, *_to_dev(torch, dev, enc)).cpu().numpy().view(np.uint64)
    bad = np.argwhere(got != want)
    print("A", A, "mismatches", len(bad), "first", bad[:6].tolist(), flush=True)
    if len(bad):
        objs = np.unique(bad[:, 0]); atts = np.unique(bad[:, 1])
        print("  objs", objs[:20].tolist(), "attrs", atts[:20].tolist(), "zeros in got", int((got[tuple(bad.T)] == 0).sum()))
