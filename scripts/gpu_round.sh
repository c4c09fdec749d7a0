#!/bin/bash
# One full GPU validation + measurement pass (run under gpurun):
#   parity tests, default bench (cfg3a, host path, cpu baseline), bench of the
#   other configs, profiles (trace + PMC traffic) for cfg3a/cfg3b, and a
#   2-rank gloo rehearsal of the multi-GPU bench flow on the one GPU.
#   bash scripts/gpu_round.sh TAG
TAG=${1:-r1}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/round_$TAG
mkdir -p $O
cd $ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench_cfg3a.json 2> $O/bench_cfg3a.err || exit $?
for c in cfg3b cfg2 cfg1; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 5 --no-host-path > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
done
bash scripts/gpu_profile.sh $TAG cfg3a || exit $?
bash scripts/gpu_profile.sh $TAG cfg3b || exit $?
HDX_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --objects 2000000 \
    > $O/bench_gloo2.json 2> $O/bench_gloo2.err || exit $?
echo "round $TAG done"
