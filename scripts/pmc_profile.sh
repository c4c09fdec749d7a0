#!/bin/bash
# SQ/TCC counter passes over scripts/run_kernel.py (run under gpurun).
#   bash scripts/pmc_profile.sh TAG CONFIG VARIANT
# PMC_SETS="A B C;D E" overrides the counter passes (';' separates passes).
TAG=${1:-pmc}; CFG=${2:-cfg3a}; VAR=${3:-12}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_${TAG}_${CFG}_v${VAR}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
RUN="$ROOT/scripts/run_kernel.py --config $CFG --variant $VAR --launches 2"
SETS=${PMC_SETS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE;SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"}
i=0
IFS=';' read -ra PASSES <<< "$SETS"
for set in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv \
      -- python3 $RUN > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "pmc $TAG $CFG v$VAR done"
