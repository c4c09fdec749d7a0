#!/bin/bash
# Wave-staged kernel: shapes A/B and counters (run under gpurun).
#   bash scripts/ws_pmc.sh TAG VARIANTS PMC_VARIANTS
TAG=${1:-ws}; VARS=${2:-44,205,207,208}; PV=${3:-"44 205"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
cd $ROOT
timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b,u150 --variants=$VARS --check 44,205 --reps 5 > $O/ab.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab.jsonl
export PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY;TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum"
for v in $PV; do
  bash scripts/pmc_profile.sh $TAG cfg3b $v > /dev/null || { echo "pmc $v failed"; exit 1; }
  echo "== cfg3b v$v"; python scripts/pmc_summary.py gpurun_out/pmc_${TAG}_cfg3b_v$v | tee $O/pmc_cfg3b_v$v.txt
done
echo "ws_pmc $TAG done"
