#!/bin/bash
# The pass-boundary gap (class_sort): every GPU test, then interleaved A/B
# against the same kernels without it (219 / 236).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-r3l}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b --variants=219,212 --reps 7 > $O/ab_3b.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab_3b.jsonl
timeout -k 10 300 python scripts/ab_variants.py --configs cfg5 --variants=236,230 --reps 7 > $O/ab_5.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab_5.jsonl
