#!/bin/bash
# Wave-staged kernel probe (run under gpurun): parity of the staged forms,
# then A/B against variant 44 on config 3b.
mkdir -p gpurun_out/ws4
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "wave_staged or (every_kernel_variant and (205 or 210 or 211))" > gpurun_out/ws4/pytest.log 2>&1 || { tail -5 gpurun_out/ws4/pytest.log; exit 1; }
tail -1 gpurun_out/ws4/pytest.log
timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b --variants=44,205,210,211 --reps 5 > gpurun_out/ws4/ab.jsonl 2> gpurun_out/ws4/ab.err || { tail -3 gpurun_out/ws4/ab.err; exit 1; }
cat gpurun_out/ws4/ab.jsonl
