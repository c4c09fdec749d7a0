#!/bin/bash
# Where the sweep's time goes: the product (230) vs its debug shapes without
# the hash (237) and without hash and walk (238); batch 212 vs 218 likewise.
set -o pipefail

ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-r3n}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_encoded.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/ab_variants.py --configs cfg5 --variants=49,230,242 --reps 7 > $O/ab_5.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab_5.jsonl


timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b --variants=212,242 --reps 9 > $O/ab_3b.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab_3b.jsonl
