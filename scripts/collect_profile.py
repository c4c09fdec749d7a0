"""Copy one evidence run (scripts/profile_r2.sh's gpurun_out/profround_TAG) into
profiles/rN: per config the bench line run under rocprofv3 --kernel-trace
(<cfg>_bench_under_rocprof.json, the JSON line only) and its kernel summary
(<cfg>_kernel_stats.csv), the default command's as default_*, and the PMC
summary traffic.json (with its source digest).

    python scripts/collect_profile.py gpurun_out/profround_r5e profiles/r5
"""
import json
import os
import shutil
import sys


def last_json_line(path):
    for line in reversed(open(path).read().splitlines()):
        line = line.strip()
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit("no JSON line in %s" % path)


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    for name in sorted(os.listdir(src)):
        if not name.endswith("_trace"):
            continue
        cfg = name[:-len("_trace")]
        bench = os.path.join(src, cfg + "_bench.json")
        stats = os.path.join(src, name, "run_kernel_stats.csv")
        if not (os.path.exists(bench) and os.path.exists(stats)):
            continue
        label = "default_bench" if cfg == "default" else cfg
        json.dump(last_json_line(bench), open(os.path.join(dst, label + "_under_rocprof.json" if cfg == "default"
                                                         else label + "_bench_under_rocprof.json"), "w"))
        shutil.copy(stats, os.path.join(dst, label + "_kernel_stats.csv"))
    t = os.path.join(src, "traffic.json")
    if os.path.exists(t):
        shutil.copy(t, os.path.join(dst, "traffic.json"))
    print(sorted(os.listdir(dst)))


if __name__ == "__main__":
    main(*sys.argv[1:3])
