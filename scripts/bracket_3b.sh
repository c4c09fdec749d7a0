#!/bin/bash
# Config 3b's line alone vs inside the default line (after the 3a headline),
# alternated twice in one call (run under gpurun): tells an in-process effect
# of the default line's order apart from the box's state.  Round 6: 2.470 /
# 2.450 / 2.455 / 2.434 ms — no difference on one box.
set -o pipefail
O=gpurun_out/bracket; mkdir -p $O
X="--no-host-path --no-stream-probe --config4-objects 0 --cpu-seconds 1 --no-cpu-baseline --no-regions"
timeout -k 10 200 python3 bench.py --config cfg3b --no-secondary $X > $O/a.json 2>/dev/null || exit 1
timeout -k 10 300 python3 bench.py --cfg5-objects 0 $X > $O/b.json 2>/dev/null || exit 1
timeout -k 10 200 python3 bench.py --config cfg3b --no-secondary $X > $O/c.json 2>/dev/null || exit 1
timeout -k 10 300 python3 bench.py --cfg5-objects 0 $X > $O/d.json 2>/dev/null || exit 1
python3 - <<'P'
import json
for f in "abcd":
    d=json.load(open("gpurun_out/bracket/%s.json"%f))
    if d["config"]["workload"].startswith("config 3b"):
        print(f, "standalone 3b", d["roofline"]["kernel_ms"], d["roofline"]["frac"])
    else:
        s=d["secondary"]["cfg3b"]; print(f, "default: 3a", d["roofline"]["kernel_ms"], "3b", s["kernel_ms"], s["roofline_frac"])
P
