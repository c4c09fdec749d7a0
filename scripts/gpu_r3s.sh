#!/bin/bash
# Regions scratch from the library's pool: regions / encoded / capi tests, then
# the regions entry points without coordinates at bench.py's sizes.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-r3s}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_regions.py tests/test_encoded.py tests/test_capi.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u scripts/ab_fused_sweep.py --batch cfg3b --objects 10000000 --variants=-1,217 --reps 7 > $O/ab.jsonl || exit 1
timeout -k 10 300 python -u scripts/ab_fused_sweep.py --objects 50000000 --variants=-1,234 --reps 3 >> $O/ab.jsonl || exit 1
cat $O/ab.jsonl
