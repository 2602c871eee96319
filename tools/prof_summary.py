"""Per-kernel duration summary from a rocprofv3 --kernel-trace run, in the layout of rocprofv3's
kernel_stats.csv (Name, Calls, TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev).

Reads either the rocpd SQLite database (rocprofv3's default output on ROCm 7.x) or a *kernel_trace.csv.
usage: python tools/prof_summary.py <results.db | kernel_trace.csv | dir> [out.csv]"""
import csv
import glob
import math
import os
import sqlite3
import sys
from collections import defaultdict


def durations(path):
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        csvs = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        path = (dbs or csvs)[0]
    per = defaultdict(list)
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        for name, start, end in con.execute("select name, start, end from kernels"):
            per[name].append(float(end - start))
    else:
        with open(path) as f:
            for row in csv.DictReader(f):
                per[row["Kernel_Name"]].append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
    return per


def main():
    per = durations(sys.argv[1])
    total = sum(sum(v) for v in per.values()) or 1.0
    rows = []
    for name, v in per.items():
        n = len(v)
        mean = sum(v) / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
        rows.append([name, n, int(sum(v)), round(mean, 3), round(100.0 * sum(v) / total, 2), int(min(v)), int(max(v)),
                     round(sd, 3)])
    rows.sort(key=lambda r: -r[2])
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    w.writerows(rows)


if __name__ == "__main__":
    main()
