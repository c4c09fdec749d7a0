# The round-end sequence the driver runs (pytest -m gpu, smoke, the default bench), in one GPU call;
# output under gpurun_out/s2w/.
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/s2w
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/s2w/tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2w/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s2w/bench.log 2> gpurun_out/s2w/bench.err || exit $?
