#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-wswp}; mkdir -p $O
export PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM"
for v in ${2:-230}; do
  bash scripts/pmc_profile.sh $1 cfg5 $v > /dev/null || { echo "pmc $v failed"; exit 1; }
  echo "== cfg5 v$v"; python scripts/pmc_summary.py gpurun_out/pmc_$1_cfg5_v$v hash_ | tee $O/pmc_cfg5_v$v.txt
  python scripts/pmc_summary.py gpurun_out/pmc_$1_cfg5_v$v sweep_ | tee -a $O/pmc_cfg5_v$v.txt
done
