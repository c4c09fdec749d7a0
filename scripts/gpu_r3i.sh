#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-r3i}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_regions.py tests/test_encoded.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "217 or regions" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in cfg3b cfg2 cfg3a; do
timeout -k 10 300 python scripts/ab_fused_sweep.py --batch $c --objects 10000000 --variants=-1,217 --reps 5 >> $O/ab.jsonl 2>> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
done
cat $O/ab.jsonl
