#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-wsw1}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_encoded.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "230 or 231 or 232" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/ab_variants.py --configs cfg5 --variants=12,230,231,232 --reps 5 > $O/ab.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab.jsonl
