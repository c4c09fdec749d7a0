#!/bin/bash
# Pass loop not unrolled (244) against the products (212 batch, 230 sweep).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-r3t}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_encoded.py tests/test_gpu_parity.py tests/test_capi.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b --variants=246,212 --reps 9 > $O/ab_3b.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab_3b.jsonl
timeout -k 10 300 python scripts/ab_variants.py --configs cfg5 --variants=246,230 --reps 9 > $O/ab_5.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab_5.jsonl
