"""Summarise rocprofv3 --pmc CSVs of one kernel: mean counter value per dispatch.
    python scripts/pmc_summary.py gpurun_out/pmc_TAG_CFG_vV [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else "hash_"
vals = defaultdict(list)
dur = []
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if ksub not in row["Kernel_Name"]:
            continue
        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
        dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
out = {k: sum(v) / len(v) for k, v in vals.items()}
for k in sorted(out):
    print("%-24s %16.1f" % (k, out[k]))
w = out.get("SQ_WAVES")
if w:
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_SMEM"):
        if k in out:
            print("%-24s %10.1f per wave" % (k, out[k] / w))
if dur:
    print("dispatch ms (profiled)  %.3f" % (sum(dur) / len(dur)))
