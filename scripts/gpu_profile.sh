#!/bin/bash
# Kernel-trace + HBM counter passes of bench.py on one GPU (run under gpurun).
#   bash scripts/gpu_profile.sh TAG CONFIG [bench args...]
# Writes gpurun_out/prof_TAG_CONFIG/{trace,fetch,write}/... plus
# traffic.json (HBM bytes per launch); copy summaries to profiles/.
TAG=${1:-r1}
CFG=${2:-cfg3a}
shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_${TAG}_${CFG}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-host-path $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 $BENCH > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err" || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
    -- python3 $BENCH > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err" || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
    -- python3 $BENCH > "$OUT/bench_write.json" 2> "$OUT/bench_write.err" || exit $?
python3 $ROOT/scripts/traffic_from_pmc.py "$OUT/fetch" "$OUT/write" $CFG "$OUT/traffic.json" || exit $?
echo "profile $TAG $CFG done"
