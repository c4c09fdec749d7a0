"""bench.py's multi-rank launch: `python3 bench.py --gpus N`
with no launcher starts N rank processes itself and prints rank 0's single
JSON line with n_gpus == N.  Rehearsed on the host (HDX_BENCH_DEVICE=cpu,
gloo): launch, config 4's shard cuts and its one-collective gather, checked
row by row — no hashing (that is the GPU's, bench.py on the box)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv, env_extra=None, timeout=240):
    env = dict(os.environ, HDX_BENCH_DEVICE="cpu", HDX_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(argv), env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    return p


@pytest.mark.parametrize("world,objects,form", [(2, 200_000, "in_place"), (3, 1001, "padded"),
                                                # the driver's SCALE command at N = 8
                                                (8, 1_600_000, "in_place"), (8, 1001, "padded")])
def test_bare_bench_spawns_ranks(world, objects, form):
    p = _bench("--gpus", str(world), "--config4-objects", str(objects))
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    res = json.loads(lines[0])
    assert res["n_gpus"] == world
    c4 = res["config4"]
    assert len(c4["objects_per_rank"]) == world and sum(c4["objects_per_rank"]) == objects
    ag = c4["allgather"]
    assert ag["collectives_per_gather"] == 1 and ag["form"] == form and ag["verified"] is True


def test_world_size_must_match_gpus():
    p = _bench("--gpus", "2", env_extra={"WORLD_SIZE": "1", "RANK": "0"}, timeout=60)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr
