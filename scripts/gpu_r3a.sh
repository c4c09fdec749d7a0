#!/bin/bash
# Round-3 first GPU pass: full parity suite, wave-staged A/B on config 3b,
# default bench line.  Stops at the first failing step.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r3a
mkdir -p $O
cd $ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b --variants=44,200,205,210,211 --reps 5 > $O/ab_ws.jsonl 2> $O/ab_ws.err || { tail -3 $O/ab_ws.err; exit 1; }
cat $O/ab_ws.jsonl
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
echo "r3a done"
