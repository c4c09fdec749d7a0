#!/bin/bash
# Parity of every kernel variant, then an interleaved A/B (run under gpurun).
#   bash scripts/quick_ab.sh TAG CONFIGS VARIANTS [PMC_VARIANT PMC_CONFIG]
TAG=$1; CFGS=$2; VARS=$3; PV=$4; PC=${5:-cfg3b}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/ab_$TAG
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_encoded.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
timeout -k 10 500 python scripts/ab_variants.py --configs $CFGS --variants=$VARS --reps 5 > $O/ab.jsonl 2> $O/ab.err || exit $?
if [ -n "$PV" ]; then
  PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE;SQ_WAVE_CYCLES SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum" \
    bash scripts/pmc_profile.sh $TAG $PC $PV > $O/pmc.log 2>&1 || exit $?
  python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}_${PC}_v$PV > $O/pmc_${PC}_v$PV.txt || exit $?
fi
echo "ab $TAG done"
