#!/bin/bash
# Sweep: LOOP 3 product vs LOOP 2 (242) and the builtin DMA (243); encoded tests first.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-r3r}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_encoded.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/ab_variants.py --configs cfg5 --variants=49,230,242,243 --reps 9 > $O/ab_5.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab_5.jsonl
