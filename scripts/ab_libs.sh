mkdir -p gpurun_out/ablibs
for r in 1 2; do
for L in NEW ALL ISSUE LE16 LOOP ROR; do
  if [ $L = NEW ]; then P=""; else P=$PWD/ab_libs/$L/libhdxhash.so; fi
  HDX_LIB_PATH=$P timeout -k 10 120 python scripts/ab_variants.py --configs cfg3b --variants 35,12 --reps 3 > gpurun_out/ablibs/${L}_$r.jsonl 2>gpurun_out/ablibs/${L}_$r.err || exit 1
done
done
