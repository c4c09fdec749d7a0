#!/bin/bash
# VALU per wave of one hash kernel variant on single-regime batches (run under gpurun):
#   bash scripts/regime_costs.sh TAG VARIANT [CONFIGS]
TAG=${1:-rc}; VAR=${2:-44}; CFGS=${3:-"u8 u24 u48 u100 u150 u190 num flt cfg3b"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU"
for c in $CFGS; do
  bash $ROOT/scripts/pmc_profile.sh $TAG $c $VAR > /dev/null || exit 1
  echo "== $c v$VAR"; python $ROOT/scripts/pmc_summary.py $ROOT/gpurun_out/pmc_${TAG}_${c}_v$VAR | grep "per wave\|dispatch"
done
