#!/bin/bash
# A/B the hash kernel variants (HDX_KERNEL_VARIANT) on several configs; under gpurun.
#   bash scripts/variant_sweep.sh TAG "0 1 2 3 4" "cfg3a cfg3b cfg2"
TAG=${1:-sweep}
VARIANTS=${2:-"0 1 2 3 4"}
CONFIGS=${3:-"cfg3a cfg3b cfg2"}
OUT=gpurun_out/sweep_$TAG
mkdir -p $OUT
for c in $CONFIGS; do
  for v in $VARIANTS; do
    HDX_KERNEL_VARIANT=$v timeout -k 10 180 python bench.py --config $c --steps 10 --warmup 2 \
        --no-cpu-baseline > $OUT/${c}_v$v.json 2> $OUT/${c}_v$v.err || exit $?
  done
done
python - "$OUT" <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.load(open(f)); r = d["roofline"]
    print(os.path.basename(f), "GiB/s", d["value"], "kernel_ms", r["kernel_ms"], "frac", r["frac"])
PY
