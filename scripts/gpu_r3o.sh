#!/bin/bash
# Per-wave instruction counts: config 5's sweep (230) and its no-hash shape
# (237) beside config 3b's batch kernel (212) and its no-hash shape (218).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-r3o}; mkdir -p $O
export PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD"
for cv in "cfg5 230" "cfg5 237" "cfg3b 212" "cfg3b 218"; do
  set -- $cv
  bash scripts/pmc_profile.sh r3o $1 $2 > /dev/null || { echo "pmc $1 $2 failed"; exit 1; }
  echo "== $1 v$2"; python scripts/pmc_summary.py gpurun_out/pmc_r3o_$1_v$2 wstage_kernel | tee $O/pmc_$1_v$2.txt
done
