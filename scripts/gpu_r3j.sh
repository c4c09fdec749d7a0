#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-r3j}; mkdir -p $O
timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b --variants=212,218 --check 212 --reps 5 > $O/ab.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab.jsonl
export PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES"
for v in 218; do
bash scripts/pmc_profile.sh $1 cfg3b $v > /dev/null && python scripts/pmc_summary.py gpurun_out/pmc_$1_cfg3b_v$v | tee $O/pmc_cfg3b_v$v.txt
done
