"""bench.py's config-5 CPU baseline also checks objects spread over the whole
store (verify_encoded_spread): here on host tensors, both store layouts, and a
single flipped coordinate in the last object is caught."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.parametrize("layout", ["keycol", "records"])
def test_spread_check_catches_a_wrong_coordinate(oracle, layout):
    import torch

    import bench
    from hyperdex_amd import synth
    types, blob, base, lens = synth.make_batch_host("cfg3b", 3000, seed=9)
    keys, ko, kl, vals, vo, vl = synth.encode_store_host(types, blob, base, lens, layout=layout)
    want, _, bad = oracle.hash_encoded(types, keys, ko, kl, vals, vo, vl)
    assert not bad.any()

    def t(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a).view(dt))
    k = t(keys, np.uint8)
    v = k if layout == "records" else t(vals, np.uint8)
    enc = (k, t(ko.astype(np.uint64), np.int64), t(kl.astype(np.uint32), np.int32), v,
           t(vo.astype(np.uint64), np.int64), t(vl.astype(np.uint32), np.int32))
    coords = torch.from_numpy(want.view(np.int64).copy())
    assert bench.verify_encoded_spread(types, enc, coords, oracle) > 64
    coords[2999, 3] ^= 1
    with pytest.raises(SystemExit):
        bench.verify_encoded_spread(types, enc, coords, oracle)
