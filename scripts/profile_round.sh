#!/bin/bash
# Evidence for the round's bench line (run under gpurun):
#  1. rocprofv3 --kernel-trace --stats of the exact default command
#     (`python3 bench.py`), whose hash-kernel average must match the bench
#     line's roofline.kernel_ms;
#  2. FETCH_SIZE / WRITE_SIZE passes (separate runs, no tracing domains) per
#     config -> traffic.json (HBM bytes per launch, gfx950 read correction).
#   bash scripts/profile_round.sh TAG "cfg3a cfg3b cfg2 cfg1 cfg5"
TAG=${1:-r1}
CFGS=${2:-"cfg3a cfg3b cfg2 cfg1 cfg5"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/profround_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/default_trace" -o run --output-format csv \
    -- python3 $ROOT/bench.py > "$OUT/default_bench.json" 2> "$OUT/default_bench.err" || exit $?
for CFG in $CFGS; do
  bash $ROOT/scripts/gpu_profile.sh $TAG $CFG || exit $?
  cp "$ROOT/gpurun_out/prof_${TAG}_${CFG}/traffic.json" "$OUT/traffic_$CFG.json" || exit $?
done
echo "profile round $TAG done"
