#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/${1:-r3g}; mkdir -p $O
timeout -k 10 120 tools/ldsbench > $O/ldsbench.jsonl 2>&1; cat $O/ldsbench.jsonl
timeout -k 10 600 python -u -m pytest tests/test_encoded.py tests/test_regions.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "encoded or regions or 216" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/ab_variants.py --configs cfg3b --variants=212,216 --reps 5 > $O/ab.jsonl 2> $O/ab.err || { tail -3 $O/ab.err; exit 1; }
cat $O/ab.jsonl
timeout -k 10 400 python bench.py --config cfg5 --no-host-path --no-stream-probe --config4-objects 0 --cpu-seconds 3 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { tail -3 $O/bench_cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_cfg5.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'], d.get('fused_regions'), d.get('regions'))"
