#!/bin/bash
# A/B the in-tree library against another build of it (run under gpurun):
#   bash scripts/ab_lib_vs.sh TAG OTHER_LIB CONFIGS VARIANTS
# Alternates the two libraries twice; each run is an interleaved A/B of the
# variants within one process (scripts/ab_variants.py).
TAG=$1; OTHER=$2; CFGS=$3; VARS=$4
O=gpurun_out/ablib_$TAG
mkdir -p $O
for r in 1 2; do
  for L in new other; do
    if [ $L = new ]; then P=""; else P=$OTHER; fi
    HDX_LIB_PATH=$P timeout -k 10 200 python scripts/ab_variants.py --configs $CFGS --variants=$VARS --reps 3 \
        > $O/${L}_$r.jsonl 2> $O/${L}_$r.err || exit 1
  done
done
echo "ablib $TAG done"
