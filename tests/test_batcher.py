"""Daemon batching shim (hdx_batcher_*): concurrent callers of
key_state::hash_objects coalesced into device batches.  tests/cpp/batcher_test.cc
drives it from many threads and checks every coordinate and region id against
the oracle; here we build it (CPU) and run it under several batch shapes (GPU)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "batcher_test")


def build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"])
    subprocess.check_call([
        "g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-pthread",
        "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle"),
        os.path.join(ROOT, "tests", "cpp", "batcher_test.cc"), "-o", EXE,
        "-L", os.path.join(ROOT, "hyperdex_amd"), "-lhdxhash",
        "-L", os.path.join(ROOT, "oracle"), "-loracle",
        "-Wl,-rpath," + os.path.join(ROOT, "hyperdex_amd") + ":" + os.path.join(ROOT, "oracle")])


def test_batcher_test_builds():
    build()
    assert os.path.exists(EXE)


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    # device batches (HDX_BATCHER_DEVICE_ONLY = 2)
    ("16", "1500", "0", "0", "0", "2"),      # defaults: 4096 objects, 4 slots, 50 us
    ("8", "600", "7", "2", "10", "2"),       # tiny batches, two slots: constant sealing/reuse
    ("1", "200", "0", "0", "2000", "2"),     # one caller: every batch ships on the deadline
    ("48", "300", "64", "3", "100", "2"),    # more callers than a batch holds
    ("16", "800", "0", "0", "0", "3"),       # staged through HBM (| HDX_BATCHER_STAGE_DEVICE)
    # the calling thread (default: objects up to 256 KiB), and a split at 300 bytes
    ("16", "1500", "0", "0", "0", "0"),
    ("16", "1500", "0", "0", "0", "0", "300"),
])
def test_batcher_concurrent_callers_match_oracle(args):
    build()
    r = subprocess.run([EXE, *args], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "batcher ok" in r.stdout
    host = int(r.stdout.split(" host ")[1].split()[0])
    batches = int(r.stdout.split(" batches ")[1].split()[0])
    if args[5] in ("2", "3"):
        assert host == 0 and batches > 0, r.stdout       # everything on the device
    elif len(args) == 6:
        assert host > 0 and batches == 0, r.stdout       # everything on the calling threads
    else:
        assert host > 0 and batches > 0, r.stdout        # split by size


@pytest.mark.gpu
def test_batcher_python_threads_match_oracle(oracle):
    """The Python wrapper from 8 threads: every object equals the oracle."""
    import threading

    import numpy as np

    import hyperdex_amd as hdx
    types = [9217, 9218, 9219, 9217, 9474]
    lo, up = oracle.partition(1, 64)
    table = hdx.RegionTable([0], lo, up, np.arange(1, 65, dtype=np.uint64))
    errors = []
    with hdx.Batcher(types, tables=[table], max_delay_us=200, host_max_bytes=100) as b:
        def worker(t):
            rng = np.random.default_rng(t)
            for _ in range(150):
                key = bytes(rng.integers(0, 256, int(rng.integers(0, 120)), dtype=np.uint8))
                vals = [bytes(rng.integers(0, 256, 8, dtype=np.uint8)) for _ in range(2)]
                vals.append(bytes(rng.integers(0, 256, int(rng.integers(0, 70)), dtype=np.uint8)))
                vals.append(bytes(rng.integers(0, 256, 8, dtype=np.uint8)))
                hs, rid = b.hash_object(key, vals)
                want = [oracle.hash_value(t_, v)[0] for t_, v in zip(types, [key] + vals)]
                wr = oracle.lookup_region([0], lo, up, np.arange(1, 65, dtype=np.uint64),
                                          np.array([want], np.uint64))[0]
                if hs != want or rid != [wr]:
                    errors.append((t, hs, want, rid, wr))
        th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        st = b.stats()
    table.close()
    assert not errors, errors[:2]
    assert st["objects"] == 8 * 150 and st["batches"] >= 1 and st["host"] >= 1
