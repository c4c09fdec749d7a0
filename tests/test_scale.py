"""The product at BASELINE's full sizes (Missing #2): paths whose
size matters — 64-bit value offsets far past 4 GiB, the regions entry
points' scratch chunks, the 100 M-object config-4 batch and its gather — are
checked here, with sampled oracle parity plus size-independent properties
(determinism across launches, equality of two independent paths).

  * config 5, the reindex sweep: 50 M stored config-3b objects (~58 GB of
    values) through hdx_hash_encoded_device and, with coords NULL,
    hdx_hash_encoded_regions_device (1 GiB scratch chunks); reference
    daemon/datalayer_encodings.cc:168-217;
  * config 4 at N = 1: 100 M config-3b objects (~109 GB) through
    dist.hash_sharded on a world-1 RCCL process group, and through the C-ABI
    device set (hdx_hash_batch_device_multi, RCCL gather); reference
    common/hash.cc:56-68.

Sampled objects: the first and last 64, those around every regions scratch
chunk edge, those whose values straddle every 4 GiB boundary of the store,
and 4 000 random ones."""
import os
import socket

import numpy as np
import pytest

import hyperdex_amd as hdx
from hyperdex_amd import dist as hdist, synth

pytestmark = pytest.mark.gpu
GiB = 1 << 30


def _gather_slices(torch, buf, off, ln):
    """Concatenate buf[off[k] : off[k] + ln[k]) for device index tensors;
    returns (host bytes, host offsets of each slice)."""
    ln = ln.to(torch.int64)
    starts = torch.cumsum(ln, 0) - ln
    total = int(ln.sum().item())
    idx = torch.repeat_interleave(off.to(torch.int64) - starts, ln) + torch.arange(total, device=buf.device)
    data = buf[idx].cpu().numpy() if total else np.zeros(1, np.uint8)
    return data, starts.cpu().numpy().view(np.uint64)


def _sample(n, extra):
    rng = np.random.default_rng(7)
    idx = np.concatenate([np.arange(64), n - 1 - np.arange(64), rng.choice(n, 4000, replace=False)] +
                         [np.asarray(e, np.int64) for e in extra])
    return np.unique(idx[(idx >= 0) & (idx < n)])


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available()
    return torch, torch.device("cuda", 0)


@pytest.mark.parametrize("layout", ["columns", "keycol", "records"])
def test_cfg5_sweep_at_50M(oracle, torch_dev, layout):
    """Config 5 at BASELINE size: 50 M stored objects, values far past 4 GiB
    of offsets; coordinates, versions and the status word sampled against
    the oracle, two launches identical, and the regions entry point with no
    coordinates (its 1 GiB scratch chunks) equal to lookups on the sweep's
    own coordinates.  Every store layout: keys in place in their packed
    objects beside a value column, a key column beside a value column, and
    records [key][value] in one store."""
    from hyperdex_amd import RegionTable
    torch, dev = torch_dev
    n = 50_000_000
    types, keys, key_off, key_len, vals, val_off, val_len = synth.make_encoded_device("cfg3b", n, device=dev,
                                                                                      layout=layout)
    A = len(types)
    assert vals.numel() > 12 * (4 * GiB)  # ~58 GB: offsets well past 2^32
    versions = torch.zeros(n, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    c1 = hdx.hash_encoded(types, keys, key_off, key_len, vals, val_off, val_len, versions=versions, status=status)
    c2 = hdx.hash_encoded(types, keys, key_off, key_len, vals, val_off, val_len)
    torch.cuda.synchronize()
    assert torch.equal(c1, c2), "two sweeps differ"
    del c2
    assert int(status.item()) == 0
    # objects whose value straddles each 4 GiB boundary of the value store
    edges = torch.arange(4 * GiB, vals.numel(), 4 * GiB, device=dev, dtype=torch.int64)
    straddle = (torch.searchsorted(val_off, edges, right=True) - 1).cpu().numpy()
    chunk = int(hdx.lib().hdxdbg_region_chunk_objects(n, A))  # objects per regions scratch chunk
    assert chunk < n
    chunk_edges = [k * chunk + d for k in range(1, n // chunk + 1) for d in (-2, -1, 0, 1)]
    idx = _sample(n, [straddle, straddle + 1, chunk_edges])
    ti = torch.from_numpy(idx).to(dev)
    assert (val_off[ti[-1]] > 8 * GiB).item()
    kb, ko = _gather_slices(torch, keys, key_off[ti], key_len[ti])
    vb, vo = _gather_slices(torch, vals, val_off[ti], val_len[ti])
    want, wver, bad = oracle.hash_encoded(types, kb, ko, key_len[ti].cpu().numpy().view(np.uint32), vb, vo,
                                          val_len[ti].cpu().numpy().view(np.uint32))
    assert not bad.any()
    assert np.array_equal(c1[ti].cpu().numpy().view(np.uint64), want)
    assert np.array_equal(versions[ti].cpu().numpy().view(np.uint64), wver)
    # regions with coords NULL (scratch chunks) == lookups of the sweep's coordinates
    specs = [([0],) + tuple(oracle.partition(1, 64)), ([1, 2, 3],) + tuple(oracle.partition(3, 64))]
    tables = [RegionTable(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 3) for at, lo, up in specs]
    ids = hdx.hash_encoded_regions(types, keys, key_off, key_len, vals, val_off, val_len, tables)
    for k, t in enumerate(tables):
        direct = hdx.lookup_region(t, c1)
        torch.cuda.synchronize()
        assert torch.equal(ids[k], direct), k
        at, lo, up = specs[k]
        w = oracle.lookup_region(at, lo, up, np.arange(1, len(lo) + 1, dtype=np.uint64) * 3, want)
        assert np.array_equal(ids[k][ti].cpu().numpy().view(np.uint64), w), k
    for t in tables:
        t.close()
    del keys, key_off, key_len, vals, val_off, val_len, c1, ids, versions
    torch.cuda.empty_cache()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_cfg4_at_N1_100M(oracle, torch_dev):
    """Config 4 at N = 1: the 100 M-object config-3b batch (~109 GB in HBM)
    through dist.hash_sharded on a world-1 RCCL process group (hash into the
    full matrix + the in-place all_gather_into_tensor), and through the C-ABI
    device set (hdx_hash_batch_device_multi with its RCCL gather): both
    identical, sampled against the oracle."""
    import torch.distributed as tdist
    torch, dev = torch_dev
    n = 100_000_000
    types, blob, base, lens = synth.make_batch_device("cfg3b", n, device=dev)
    A = len(types)
    assert blob.numel() > 100 * GiB
    sizes = lens.view(n, A).to(torch.int64).sum(dim=1)
    ranges = hdist.shard_ranges(n, 1, sizes, equal_count_tol=1e-3)
    del sizes
    assert ranges == [(0, n)]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    tdist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        full = hdist.hash_sharded(types, blob, base, lens, [n])
        torch.cuda.synchronize()
    finally:
        tdist.destroy_process_group()
    assert full.shape == (n, A)
    hdx.init_mask(1)
    try:
        (multi,) = hdx.hash_batch_device_multi(types, [(blob, base, lens)], gather=True)
    finally:
        hdx.shutdown()
    assert torch.equal(full, multi), "hash_sharded and the C-ABI device set differ"
    del multi
    idx = _sample(n, [])
    ti = torch.from_numpy(idx).to(dev)
    sl = lens.view(n, A)[ti]
    bb, bo = _gather_slices(torch, blob, base[ti], sl.to(torch.int64).sum(dim=1))
    want, err = oracle.hash_batch(types, bb, bo, sl.cpu().numpy().view(np.uint32).ravel())
    assert err == 0
    assert np.array_equal(full[ti].cpu().numpy().view(np.uint64), want)
    del blob, base, lens, full
    torch.cuda.empty_cache()
