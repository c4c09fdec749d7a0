#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/ws2; mkdir -p $O
timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b --variants=205,200,201,204,210,211 --reps 5 > $O/ab.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab.jsonl
export PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
for v in 210 204 201; do
  bash scripts/pmc_profile.sh ws2 cfg3b $v > /dev/null || { echo "pmc $v failed"; exit 1; }
  echo "== cfg3b v$v"; python scripts/pmc_summary.py gpurun_out/pmc_ws2_cfg3b_v$v | tee $O/pmc_cfg3b_v$v.txt
done
