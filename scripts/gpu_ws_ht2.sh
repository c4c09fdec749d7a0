#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-ht2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "(every_kernel_variant and 215) or (wave_staged and 215)" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b --variants=44,212,215 --reps 5 > $O/ab.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab.jsonl
bash scripts/regime_costs.sh rc13 213 "u8 u24 u48 u100 u150 num flt cfg3b" > $O/regime_costs_v213.txt 2>&1 || { tail $O/regime_costs_v213.txt; exit 1; }
cat $O/regime_costs_v213.txt
