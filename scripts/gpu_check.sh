#!/bin/bash
# Quick GPU pass (run under gpurun): build, full parity suite, the batcher's
# throughput/latency sweep, the default bench line, and an interleaved A/B of
# kernel variants on config 3b / config 5.  Stops at the first failing step.
#   bash scripts/gpu_check.sh TAG [VARIANTS_3B]
TAG=${1:-check}
V3B=${2:-44,38,35,12}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/check_$TAG
mkdir -p $O
cd $ROOT
make -s -j8 -C hyperdex_amd/csrc > $O/build.log 2>&1 || exit $?
make -s -C tools batcher_bench >> $O/build.log 2>&1 || exit $?
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in "1 2 0 0 3 0" "1 2 0 0 3 1" "16 3 0 0 3 0" "16 3 0 0 3 1" "64 3 0 0 3 0" "256 3 0 0 3 0" "16 3 0 0 0 0"; do
  timeout -k 10 60 tools/batcher_bench $cfg >> $O/batcher_bench.jsonl 2>> $O/batcher_bench.err || exit $?
done
timeout -k 10 300 python bench.py --cpu-seconds 5 > $O/bench_cfg3a.json 2> $O/bench_cfg3a.err || exit $?
timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b --variants=$V3B --reps 5 > $O/ab_cfg3b.jsonl 2> $O/ab_cfg3b.err || exit $?
echo "check $TAG done"
