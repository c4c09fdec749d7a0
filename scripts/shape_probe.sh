#!/bin/bash
# Memory-only / arithmetic-only shapes of the chunk kernel (variants 40/41)
# next to the real one (12), with TA/SQ counters (run under gpurun).
#   bash scripts/shape_probe.sh TAG
TAG=${1:-shape}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/shape_$TAG
mkdir -p $O
cd $ROOT
timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b,cfg3a --variants 12,40,41 --reps 5 > $O/ab.jsonl 2> $O/ab.err || exit $?
for v in 12 40 41; do
  PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
    bash scripts/pmc_profile.sh $TAG cfg3b $v > $O/pmc_$v.log 2>&1 || exit $?
  python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_cfg3b_v$v > $O/pmc_cfg3b_v$v.txt || exit $?
done
echo "shape $TAG done"
