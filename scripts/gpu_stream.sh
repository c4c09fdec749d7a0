#!/bin/bash
# streamed kernel: parity, then A/B against the product kernels (run under gpurun)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-st1}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "stream_kernel or (every_kernel_variant and (220 or 221 or 222)) or (wave_staged and (220 or 221 or 222))" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python scripts/ab_variants.py --configs ${3:-cfg3b,cfg3a,cfg2,cfg1} --variants=${2:-44,220,221,222,223,224,225} --check 44,220,221,222 --reps 3 > $O/ab.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab.jsonl
