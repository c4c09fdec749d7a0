#!/bin/bash
# wave-staged shapes + counters, then config 2's drift probe
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
bash scripts/ws_pmc.sh ws1 || exit $?
mkdir -p gpurun_out/drift
timeout -k 10 200 python scripts/drift_probe.py --config cfg2 --launches 40 > gpurun_out/drift/cfg2.jsonl 2> gpurun_out/drift/cfg2.err || { tail -3 gpurun_out/drift/cfg2.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/drift/cfg2.jsonl"):
    d = json.loads(l)
    d.pop("kernel_ms", None)
    print(d)
PY
