#!/bin/bash
# Round evidence (run under gpurun), everything under gpurun_out/profround_TAG:
#  1. rocprofv3 --kernel-trace --stats of the exact default command
#     (`python3 bench.py`): its hash-kernel average must agree with the bench
#     line's roofline.kernel_ms;
#  2. per config, the bench line under --kernel-trace --stats (config 5 at
#     BASELINE's 50 M objects);
#  3. per config, FETCH_SIZE and WRITE_SIZE in separate --pmc runs of
#     scripts/run_kernel.py (the product kernel alone) -> traffic.json with
#     the kernel-source digest bench.py checks.
#   bash scripts/profile_r2.sh TAG
#   bash scripts/profile_r2.sh TAG [trace|pmc|all]   (default all; each part fits one GPU call)
TAG=${1:-r2}
MODE=${2:-all}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/profround_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
if [ "$MODE" != pmc ]; then
echo "[$(date +%T)] default bench under kernel trace"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/default_trace" -o run --output-format csv \
    -- python3 $ROOT/bench.py > "$OUT/default_bench.json" 2> "$OUT/default_bench.err" || exit $?
for CFG in cfg3b cfg2 cfg1 cfg5 cfg5k cfg5r; do
  echo "[$(date +%T)] $CFG bench under kernel trace"
  EXTRA="--no-secondary --no-host-path --no-stream-probe --config4-objects 0 --cpu-seconds 3"
  B=$CFG
  case $CFG in cfg5k) B="cfg5 --store-layout keycol";; cfg5r) B="cfg5 --store-layout records";; esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/${CFG}_trace" -o run --output-format csv \
      -- python3 $ROOT/bench.py --config $B $EXTRA > "$OUT/${CFG}_bench.json" 2> "$OUT/${CFG}_bench.err" || exit $?
done
fi
[ "$MODE" = trace ] && { echo "profile round $TAG (trace) done"; exit 0; }
for CFG in cfg3a cfg3b cfg2 cfg1 cfg5 cfg5k cfg5r; do
  N=10000000; case $CFG in cfg5*) N=50000000;; esac
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "[$(date +%T)] $CFG $C"
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/pmc_${CFG}_$C" -o run --output-format csv \
        -- python3 $ROOT/scripts/run_kernel.py --config $CFG --launches 3 --objects $N \
        > "$OUT/pmc_${CFG}_$C.log" 2>&1 || exit $?
  done
  # the VALU-issue roofline's counters (4 SQ + 1 GRBM: one pass), with the
  # kernel trace for the effective clock
  echo "[$(date +%T)] $CFG VALU"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE \
      -d "$OUT/pmc_${CFG}_VALU" -o run --output-format csv \
      -- python3 $ROOT/scripts/run_kernel.py --config $CFG --launches 3 --objects $N \
      > "$OUT/pmc_${CFG}_VALU.log" 2>&1 || exit $?
  python3 $ROOT/scripts/traffic_from_pmc.py "$OUT/pmc_${CFG}_FETCH_SIZE" "$OUT/pmc_${CFG}_WRITE_SIZE" $CFG \
      "$OUT/traffic.json" $N "$OUT/pmc_${CFG}_VALU" || exit $?
done
echo "profile round $TAG done"
