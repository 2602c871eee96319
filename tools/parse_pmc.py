"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch) and derive HBM bytes per launch of the roofline
kernels.  FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE
under-reports wide coalesced reads by 2x; k_batch_integrate's access widths are not the calibrated 16-B streaming
pattern, so its read side is calibrated on k_export (bench.py --calib), whose reads have the integrate kernel's
exact 4-B-per-lane row pattern over the voxel pool and a known byte count (80 KiB per unit).  Other kernels use the
guide's 2x.  The output is tagged with the build's source hash and the workload, and bench.py uses it only when both
match."""
import csv
import glob
import importlib
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ROOF = ("k_batch_integrate", "k_sor_knn")


def load(dirs):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    short = row.get("Kernel_Name", "").split("(")[0].split("::")[-1].split("<")[0]
                    per[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


def main():
    dirs = sys.argv[1:]
    per = load(dirs)
    summary = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}
    L = importlib.import_module("object-triggered-3d-slam_amd._lib")
    units = None
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*.log")) + [d + ".log"]:
            if os.path.exists(f):
                for line in open(f):
                    if line.startswith("{") and '"volume_units"' in line:
                        units = json.loads(line)["config"]["volume_units"]
    exp = summary.get("k_export", {})
    calib = (units * 81920.0) / (exp["FETCH_SIZE"] * 1024.0) if (exp.get("FETCH_SIZE") and units) else None
    out = {"source_hash": L.source_hash(), "config": {"voxel": 0.005, "frames": 256, "batch": 0},
           "kernels_traffic": {}, "kernels": summary}
    for kern in ROOF:
        k = summary.get(kern, {})
        if k.get("FETCH_SIZE") is None or k.get("WRITE_SIZE") is None:
            continue
        corr = calib if (kern == "k_batch_integrate" and calib) else 2.0
        fetch = k["FETCH_SIZE"] * 1024.0 * corr
        write = k["WRITE_SIZE"] * 1024.0
        ent = {"bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch), "write_bytes": round(write),
               "fetch_correction": corr, "raw_fetch_kib": k["FETCH_SIZE"], "raw_write_kib": k["WRITE_SIZE"]}
        if k.get("SQ_WAVE_CYCLES"):
            wc = k["SQ_WAVE_CYCLES"]
            ent["stall_shares"] = {"wait_any": k.get("SQ_WAIT_ANY", 0) / wc, "wait_inst_any": k.get("SQ_WAIT_INST_ANY", 0) / wc,
                                   "active_inst_any": k.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                                   "active_valu": k.get("SQ_ACTIVE_INST_VALU", 0) / wc}
        if k.get("SQ_ACTIVE_INST_VALU") and k.get("GRBM_GUI_ACTIVE"):
            # VALU issue: wave-cycles with a VALU instruction in flight (quad-cycle counter x 4) per SIMD-cycle of
            # the dispatch (GRBM_GUI_ACTIVE sums the 8 XCDs' cycles; MI355X_MICROARCH.md): the roofline of a kernel
            # bound by vector-ALU issue rather than by bytes
            cyc = k["GRBM_GUI_ACTIVE"] / 8.0
            ent["valu_busy_frac"] = k["SQ_ACTIVE_INST_VALU"] * 4.0 / 1024.0 / cyc
            ent["valu_insts_per_launch"] = k.get("SQ_INSTS_VALU")
            ent["dispatch_cycles"] = cyc
        out["kernels_traffic"][kern] = ent
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
