#!/bin/bash
# Sweep: key span DMA + branch-free walk: encoded GPU tests, then A/B against
# the gather sweep (49, unchanged) as the reference.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-r3m}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_encoded.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/ab_variants.py --configs cfg5 --variants=49,236,230 --reps 7 > $O/ab_5.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab_5.jsonl
