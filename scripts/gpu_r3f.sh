#!/bin/bash
# full GPU parity suite + config-5 bench line at BASELINE's 50 M objects
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-r3f}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --config cfg5 --no-host-path --no-stream-probe --config4-objects 0 --cpu-seconds 3 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -3 $O/bench_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'], d.get('fused_regions'))"
