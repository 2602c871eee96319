#!/bin/bash
# rocprofv3 kernel-trace summary of one bench invocation: BENCH_ARGS env -> gpurun_out/prof_b/kernel_stats.csv
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b -o bench -- \
    python3 bench.py $BENCH_ARGS > gpurun_out/prof_b.log 2>&1 || { tail -30 gpurun_out/prof_b.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_b gpurun_out/prof_b/kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_b/kernel_stats.csv")))
for r in rows[:28]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
