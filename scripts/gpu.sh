#!/bin/bash
# One parameterised GPU runner (run under gpurun).  Every step runs under its
# own time limit; the first failing step ends the call.  Output goes to
# gpurun_out/<tag>/.
#
#   bash scripts/gpu.sh TAG STEP [STEP ...]
#
# Steps:
#   tests[=K]          pytest -m gpu (optionally -k K)
#   testfile=F[,F...]  pytest -m gpu on the named files only
#   smoke              __graft_entry__.smoke()
#   bench[=ARGS]       python bench.py ARGS   (ARGS: commas for spaces)
#   ab=CFG:V1,V2[:R]   scripts/ab_variants.py, interleaved A/B of debug variants
#   pmc=CFG:V1,V2[:SET] counter passes over scripts/run_kernel.py per variant (pmc_profile.sh),
#                      summarised by pmc_summary.py; SET "lds" = the LDS / VALU / wait set
#   profile[=MODE]     scripts/profile_r2.sh TAG MODE (round evidence: MODE trace | pmc | all)
#   py=SCRIPT[,ARGS]   python SCRIPT ARGS (commas for spaces)
#   sh=SCRIPT[,ARGS]   bash SCRIPT ARGS (commas for spaces)
#   exe=PROG[,ARGS]    ./PROG ARGS (a built tool; commas for spaces)
set -o pipefail
TAG=${1:?tag}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
O=gpurun_out/$TAG
mkdir -p "$O"
i=0
for STEP in "$@"; do
  i=$((i + 1))
  name=${STEP%%=*}; arg=${STEP#*=}; [ "$arg" = "$STEP" ] && arg=""
  log="$O/$(printf %02d $i)_$name.log"
  echo "[$(date +%T)] step $i: $STEP"
  case $name in
    tests)
      K=(); [ -n "$arg" ] && K=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
          -p no:cacheprovider "${K[@]}" > "$log" 2>&1 ;;
    testfile)
      timeout -k 10 900 python -u -m pytest ${arg//,/ } -m gpu -x -q --timeout 300 --timeout-method thread \
          -p no:cacheprovider > "$log" 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 ;;
    bench)
      timeout -k 10 600 python -u bench.py ${arg//,/ } > "$log" 2> "$log.err" ;;
    ab)
      IFS=: read -r cfg vars reps <<< "$arg"
      timeout -k 10 600 python -u scripts/ab_variants.py --configs "$cfg" --variants="$vars" --reps "${reps:-9}" \
          > "$log" 2> "$log.err" ;;
    pmc)
      IFS=: read -r cfg vars set <<< "$arg"
      if [ "$set" = lds ]; then
        export PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY;FETCH_SIZE;WRITE_SIZE"
      fi
      rc=0
      for v in ${vars//,/ }; do
        timeout -k 10 600 bash scripts/pmc_profile.sh "$TAG" "$cfg" "$v" >> "$log" 2>&1 || { rc=$?; break; }
        echo "== $cfg v$v" >> "$log"
        python scripts/pmc_summary.py "gpurun_out/pmc_${TAG}_${cfg}_v$v" >> "$log" 2>&1 || { rc=$?; break; }
      done
      (exit $rc) ;;
    profile)
      timeout -k 10 1150 bash scripts/profile_r2.sh "$TAG" "${arg:-all}" > "$log" 2>&1 ;;
    py)
      timeout -k 10 900 python -u ${arg//,/ } > "$log" 2> "$log.err" ;;
    sh)
      timeout -k 10 900 bash ${arg//,/ } > "$log" 2> "$log.err" ;;
    exe)
      timeout -k 10 300 ${arg//,/ } > "$log" 2> "$log.err" ;;
    *)
      echo "unknown step $STEP"; exit 2 ;;
  esac
  rc=$?
  tail -3 "$log"
  if [ $rc -ne 0 ]; then
    echo "step $i ($STEP) failed rc=$rc"
    [ -f "$log.err" ] && tail -20 "$log.err"
    tail -30 "$log"
    exit $rc
  fi
done
echo "[$(date +%T)] $TAG done"
