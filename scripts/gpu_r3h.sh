#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-r3h}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_encoded.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "regions" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --config cfg5 --no-host-path --no-stream-probe --config4-objects 0 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -3 $O/bench_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'], d.get('fused_regions'), d.get('regions'))"
