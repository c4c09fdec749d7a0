#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-ht1}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "(every_kernel_variant and (212 or 214)) or (wave_staged and (212 or 214))" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b,cfg3a --variants=44,205,212,214 --reps 5 > $O/ab.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab.jsonl
export PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
bash scripts/pmc_profile.sh $1 cfg3b 212 > /dev/null && python scripts/pmc_summary.py gpurun_out/pmc_$1_cfg3b_v212 | tee $O/pmc_cfg3b_v212.txt
