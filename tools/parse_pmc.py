"""Summarise rocprofv3 --pmc CSVs per kernel (mean per dispatch) and derive HBM bytes per launch of the roofline
kernels.  FETCH_SIZE / WRITE_SIZE are KiB per dispatch.

gfx950 corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE under-reports wide coalesced streaming reads by 2x, and other
access widths are uncalibrated.  The correction applied here is MEASURED on the access pattern it is applied to:
tools/fetch_calib.hip reads / writes a 1-GiB buffer exactly once per pattern (16-B streaming, 8-B and 4-B buffer
gathers consuming whole lines, an 8-B half-line granularity probe, 8-B buffer stores), so each pattern's factor =
known bytes / counter bytes.  k_batch_integrate's reads are 8-B buffer gathers (staged depth + multiplier; float64
colour state) and 4-B gathers (colour, float32 planes): it takes the 8-B gather factor; k_sor_knn (8-B point gathers)
too; the write side takes the 8-B store factor.  Raw counters and the factor are reported side by side.

Usage: parse_pmc.py --calib <dir>... -- <dir>...   (kernels named k_batch_integrate keep their template argument:
<true> = float64 colour, <false> = float32 colour).  The output is tagged with the build's source hash and each
entry with its workload; bench.py uses an entry only when both match."""
import csv
import glob
import importlib
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ROOF = ("k_batch_integrate<true>", "k_batch_integrate<false>", "k_sor_knn")
BASE_CFG = {"voxel": 0.005, "frames": 256, "batch": 0}


def short_name(full):
    base = full.split("(")[0].split("::")[-1]
    if base.startswith("k_batch_integrate<"):  # <C64, FAST, ZB>: the reciprocal-table coarse kernel keeps the bench's name
        args = [a.strip() for a in base[base.index("<") + 1:base.rindex(">")].split(",")]
        return f"k_batch_integrate<{args[0]}>" + ("" if len(args) < 2 or args[1] == "true" else "[ieee]") + \
            ("[fine]" if len(args) > 2 and args[2] == "2" else "")
    return base.split("<")[0]


def load(dirs):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    per[short_name(row.get("Kernel_Name", ""))][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


def filter_config(dirs):
    """workload of the configs[2] PMC runs: tools/filter_batch_time.py prints one JSON line per batch size with the
    frames per launch and the SOR kNN's algorithmic bytes per launch (12 B per input point + 12 B per kept point)"""
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*.log")) + [d + ".log"]:
            if os.path.exists(f):
                for line in open(f):
                    if line.startswith("{") and "filter_batch" in line:
                        j = json.loads(line)
                        return {"batch": j["filter_batch"], "frames": j["frames"],
                                "algorithmic_bytes_per_launch": round(j["sor_algorithmic_bytes_per_launch"])}
    return {}


def calibration(dirs):
    """Factors known bytes / counter bytes per fetch_calib pattern (None when the calibration run is missing)."""
    per = load(dirs)
    summ = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}
    known = None
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*.log")) + [d + ".log"]:
            if os.path.exists(f):
                for line in open(f):
                    if line.startswith("{") and "known_read_bytes" in line:
                        known = json.loads(line)
    if not known:
        return None
    out = {"buffer_bytes": known["buffer_bytes"], "patterns": {}}
    for k, b in known["known_read_bytes"].items():
        kern = k.replace("_used", "").replace("_lines", "")
        fs = summ.get(kern, {}).get("FETCH_SIZE")
        if fs:
            out["patterns"][k] = {"raw_fetch_kib": fs, "known_bytes": b, "factor": b / (fs * 1024.0)}
    for k, b in known["known_write_bytes"].items():
        ws = summ.get(k, {}).get("WRITE_SIZE")
        if ws:
            out["patterns"][k] = {"raw_write_kib": ws, "known_bytes": b, "factor": b / (ws * 1024.0)}
    return out


def main():
    argv = sys.argv[1:]
    calib_dirs, dirs = [], argv
    if argv and argv[0] == "--calib":
        sep = argv.index("--")
        calib_dirs, dirs = argv[1:sep], argv[sep + 1:]
    per = load(dirs)
    summary = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}
    L = importlib.import_module("object-triggered-3d-slam_amd._lib")
    cal = calibration(calib_dirs) if calib_dirs else None
    pat = (cal or {}).get("patterns", {})
    f8 = pat.get("k_cal_gather8", {}).get("factor")
    w8 = pat.get("k_cal_store8", {}).get("factor")
    out = {"source_hash": L.source_hash(), "config": BASE_CFG, "calibration": cal, "kernels_traffic": {},
           "kernels": summary}
    for kern in ROOF:
        k = summary.get(kern, {})
        if k.get("FETCH_SIZE") is None or k.get("WRITE_SIZE") is None:
            continue
        fcorr = f8 if f8 else 2.0
        wcorr = w8 if w8 else 1.0
        fetch = k["FETCH_SIZE"] * 1024.0 * fcorr
        write = k["WRITE_SIZE"] * 1024.0 * wcorr
        cfg = dict(BASE_CFG)
        if kern.startswith("k_batch_integrate"):
            cfg["color_bits"] = 64 if kern.endswith("<true>") else 32
        else:  # k_sor_knn: the configs[2] chain at the batch size the filter runs used (their logs say it)
            cfg = filter_config(dirs)
        ent = {"config": cfg, "bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch),
               "write_bytes": round(write), "fetch_correction": fcorr, "write_correction": wcorr,
               "fetch_correction_source": "tools/fetch_calib.hip k_cal_gather8 (8-B buffer gathers, measured)" if f8
               else "MI355X_MICROARCH.md 2x (16-B streaming reads; no calibration run)",
               "raw_fetch_kib": k["FETCH_SIZE"], "raw_write_kib": k["WRITE_SIZE"],
               "raw_bytes_per_launch": round((k["FETCH_SIZE"] + k["WRITE_SIZE"]) * 1024.0)}
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
        if k.get("TCC_HIT_sum") is not None and k.get("TCC_MISS_sum") is not None:
            # L2 (TCC) hit share of the kernel's requests: the misses are what FETCH_SIZE counts as fabric traffic
            h, m = k["TCC_HIT_sum"], k["TCC_MISS_sum"]
            ent["tcc_hit"], ent["tcc_miss"] = h, m
            ent["tcc_hit_frac"] = h / (h + m) if h + m > 0 else None
        if k.get("TA_TA_BUSY_sum") and k.get("GRBM_GUI_ACTIVE"):
            ent["ta_busy_frac"] = k["TA_TA_BUSY_sum"] / 256.0 / (k["GRBM_GUI_ACTIVE"] / 8.0)
            ent["td_busy_frac"] = k.get("TD_TD_BUSY_sum", 0) / 256.0 / (k["GRBM_GUI_ACTIVE"] / 8.0)
        out["kernels_traffic"][kern] = ent
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
