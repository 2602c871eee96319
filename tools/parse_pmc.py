"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch) and derive HBM traffic per launch of the
dominant kernel.  FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  gfx950 correction (MI355X_MICROARCH.md, HBM):
FETCH_SIZE under-reports wide coalesced reads by 2x; our kernels' access widths are not the calibrated 16-B
streaming pattern, so the read side is calibrated on k_export, whose reads have the integrate kernel's exact
4-B-per-lane row pattern over the voxel pool and a known byte count (80 KiB per unit)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = "k_batch_integrate"


def load(dirs):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    short = name.split("(")[0].split("::")[-1]
                    per[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


def main():
    dirs = sys.argv[1:]
    per = load(dirs)
    summary = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}
    out = {"kernels": summary}
    k = summary.get(KERNEL, {})
    exp = summary.get("k_export", {})
    units = None
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*.log")) + [d + ".log"]:
            if os.path.exists(f):
                for line in open(f):
                    if line.startswith("{") and '"volume_units"' in line:
                        units = json.loads(line)["config"]["volume_units"]
    calib = None
    if exp.get("FETCH_SIZE") and units:
        calib = (units * 81920.0) / (exp["FETCH_SIZE"] * 1024.0)
    if k.get("FETCH_SIZE") is not None and k.get("WRITE_SIZE") is not None:
        fetch = k["FETCH_SIZE"] * 1024.0 * (calib if calib else 2.0)
        write = k["WRITE_SIZE"] * 1024.0
        out.update({"kernel": KERNEL, "bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch),
                    "write_bytes": round(write), "fetch_correction": calib if calib else 2.0,
                    "raw_fetch_kib": k["FETCH_SIZE"], "raw_write_kib": k["WRITE_SIZE"]})
    if k.get("SQ_WAVE_CYCLES"):
        wc = k["SQ_WAVE_CYCLES"]
        out["stall_shares"] = {"wait_any": k.get("SQ_WAIT_ANY", 0) / wc, "wait_inst_any": k.get("SQ_WAIT_INST_ANY", 0) / wc,
                               "active_inst_any": k.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                               "active_valu": k.get("SQ_ACTIVE_INST_VALU", 0) / wc}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
