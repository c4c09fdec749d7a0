#!/bin/bash
# Traffic and instruction counters of the wide sweep's two launches (run under
# gpurun): FETCH_SIZE, WRITE_SIZE and an SQ pass per kernel, w200 key column.
#   bash scripts/pmc_wide.sh TAG [SCHEMA]
TAG=${1:-wide}; SCHEMA=${2:-w200}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
bash "$ROOT/scripts/pmc_profile.sh" "$TAG" "cfg5k_$SCHEMA" -1 || exit 1
for k in sweep_wide_walk sweep_wide_hash; do
  echo "== $k"
  python3 "$ROOT/scripts/pmc_summary.py" "$ROOT/gpurun_out/pmc_${TAG}_cfg5k_${SCHEMA}_v-1" "$k" || exit 1
done
