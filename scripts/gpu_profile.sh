#!/bin/bash
# Kernel-trace + HBM counter passes of bench.py on one GPU (run under gpurun).
#   bash scripts/gpu_profile.sh TAG [bench args...]
# Writes gpurun_out/prof_TAG/{trace,fetch,write}/...; copy summaries to profiles/.
TAG=${1:-r1}
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 $BENCH > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err" || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
    -- python3 $BENCH > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err" || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
    -- python3 $BENCH > "$OUT/bench_write.json" 2> "$OUT/bench_write.err" || exit $?
echo "profile $TAG done"
