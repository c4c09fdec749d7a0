#!/bin/bash
# Daemon batching shim under load (run under gpurun; tools/batcher_bench built
# beforehand): callers x {calling-thread default, HDX_BATCHER_DEVICE_ONLY},
# then the crossover by object size at one caller (strings scaled x1..x1024).
#   bash scripts/batcher_sweep.sh OUT.jsonl
OUT=${1:-gpurun_out/batcher_sweep.jsonl}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
: > "$OUT"
for T in 1 16 64 256; do
  for F in 0 2; do
    timeout -k 10 60 tools/batcher_bench $T 2 0 0 3 $F >> "$OUT" || exit $?
  done
done
for S in 1 16 64 256 1024; do
  # host_max_bytes huge: every object on the calling thread; flags 2: every object on the device
  timeout -k 10 60 tools/batcher_bench 1 2 0 0 3 0 1000000000 $S >> "$OUT" || exit $?
  timeout -k 10 60 tools/batcher_bench 1 2 0 0 3 2 0 $S >> "$OUT" || exit $?
done
cat "$OUT"
