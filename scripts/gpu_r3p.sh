#!/bin/bash
# The wave-staged kernel's DMA as inline asm (ADMA): parity, then A/B against
# the builtin DMA (240) and the no-hash shapes (241 ADMA, 218 builtin).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-r3p}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_capi.py tests/test_regions.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b --variants=240,212,218,241 --reps 9 > $O/ab_3b.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab_3b.jsonl
