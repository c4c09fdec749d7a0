# Multi-rank rehearsal on a one-GPU box (run under gpurun): two ranks on cuda:0 over gloo,
# the real kernels, config 4 at 20 M objects; the line lands in gpurun_out/s2u/.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/s2u
HDX_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --config4-objects 20000000 > gpurun_out/s2u/bench_gloo2.log 2> gpurun_out/s2u/bench_gloo2.err
