#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
rm -rf gpurun_out/prof_c
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c -o c -- python3 tools/chain_stats.py > gpurun_out/prof_c.log 2>&1 || { tail -20 gpurun_out/prof_c.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_c gpurun_out/prof_c/ks.csv > /dev/null
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/prof_c/ks.csv")):
    if "chain" in r["Name"]:
        print(r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", r["Name"][:60])
PY
