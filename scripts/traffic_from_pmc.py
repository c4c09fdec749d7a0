"""HBM bytes per launch of the hash kernel from rocprofv3 --pmc passes.

    python scripts/traffic_from_pmc.py FETCH_DIR WRITE_DIR CONFIG OUT_JSON [OBJECTS [VALU_DIR]]

FETCH_SIZE and WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reads exactly half
the bytes of a wide (16 B/lane) coalesced streaming read (MI355X_MICROARCH.md
§HBM); the kernel's reads are dominated by such loads, so FETCH is doubled.
Calibration: on config 3a, 2 x FETCH_SIZE equals the
algorithmic read bytes (blob + lengths + object bases) to 0.1 %.

VALU_DIR (optional): a --kernel-trace --pmc pass of SQ_INSTS_VALU,
SQ_INSTS_SALU, SQ_WAVES and GRBM_GUI_ACTIVE: per launch the vector and scalar
instructions (summed over waves), the waves, and the effective clock
GRBM_GUI_ACTIVE / 8 XCDs / kernel time (MI355X_MICROARCH.md, DVFS) — from
which bench.py reports the VALU-issue roofline of the VALU-bound kernels.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "hash_" in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit("no %s rows for the hash kernel under %s" % (counter, d))
    return sum(vals) / len(vals), len(vals)


def kernel_ns(d):
    """Mean duration of the hash kernel's dispatches in a --kernel-trace output."""
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "hash_" in row["Kernel_Name"]:
                vals.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    if not vals:
        raise SystemExit("no hash kernel dispatches in the kernel trace under %s" % d)
    return sum(vals) / len(vals)


def main(fetch_dir, write_dir, config, out, objects="10000000", valu_dir=None):
    fetch_kib, nf = per_dispatch(fetch_dir, "FETCH_SIZE")
    write_kib, nw = per_dispatch(write_dir, "WRITE_SIZE")
    rec = {"config": config, "objects": int(objects), "dispatches": [nf, nw],
           "fetch_size_kib": fetch_kib, "write_size_kib": write_kib,
           "read_bytes": 2 * fetch_kib * 1024, "write_bytes": write_kib * 1024,
           "traffic_bytes": 2 * fetch_kib * 1024 + write_kib * 1024,
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 wide-read undercount); write = WRITE_SIZE x 1024"}
    if valu_dir:
        valu, _ = per_dispatch(valu_dir, "SQ_INSTS_VALU")
        salu, _ = per_dispatch(valu_dir, "SQ_INSTS_SALU")
        waves, _ = per_dispatch(valu_dir, "SQ_WAVES")
        grbm, _ = per_dispatch(valu_dir, "GRBM_GUI_ACTIVE")
        ns = kernel_ns(valu_dir)
        rec.update({"valu_insts": valu, "salu_insts": salu, "waves": waves, "grbm_gui_active": grbm,
                    "pmc_kernel_ns": ns, "effective_clock_ghz": grbm / 8 / ns,
                    "valu_per_wave": valu / waves if waves else None,
                    "salu_per_wave": salu / waves if waves else None})
    data = {}
    if os.path.exists(out):
        data = json.load(open(out))
    # the kernel sources these counters measured (bench.py refuses other sources' traffic)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    digest = bench.source_digest()
    if data.get("source_digest") not in (None, digest):
        data = {}  # an older build's records are not this build's traffic
    data["source_digest"] = digest
    data[config] = rec
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main(*sys.argv[1:7])
