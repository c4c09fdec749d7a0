#!/bin/bash
# Regions by hash + separate lookups: parity tests, then interleaved A/B of
# the product (by lookup from 2^20 objects, 1 GiB chunks) against the fused
# forms (217 wave-staged batch, 234 gather sweep) and 235 (64 MiB chunks).
set -o pipefail
OUT=gpurun_out/r3k
mkdir -p $OUT
rm -f $OUT/ab_*.jsonl; [ -n "$SKIP_TESTS" ] ||
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_regions.py tests/test_encoded.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u scripts/ab_fused_sweep.py --batch cfg3b --objects 10000000 \
    --variants=-1,217,235 --reps 5 >> $OUT/ab_batch.jsonl || exit 1
timeout -k 10 200 python -u scripts/ab_fused_sweep.py --batch cfg2 --objects 10000000 \
    --variants=-1 --reps 5 >> $OUT/ab_batch.jsonl || exit 1
cat $OUT/ab_batch.jsonl
timeout -k 10 300 python -u scripts/ab_fused_sweep.py --objects 50000000 \
    --variants=-1,234,235 --reps 3 >> $OUT/ab_sweep.jsonl || exit 1
cat $OUT/ab_sweep.jsonl
