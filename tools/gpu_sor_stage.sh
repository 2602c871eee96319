#!/bin/bash
# SOR change check on one GPU box: SOR / filter-chain parity tests, then the configs[2] batch chain's kernel
# breakdown (rocprofv3 --kernel-trace --stats of tools/filter_batch_time.py, 32-frame batches).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-sor}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_filters.py tests/test_gpu_filter_batch.py} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o fb -- python3 tools/filter_batch_time.py --frames ${FRAMES:-64} --batches 32 > gpurun_out/${TAG}_fbt.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/${TAG}_fbt.log; exit 1; }
grep "batch 32" gpurun_out/${TAG}_fbt.log
python3 tools/prof_summary.py gpurun_out/${TAG}_prof gpurun_out/${TAG}_prof/kernel_stats.csv > /dev/null
python3 - <<PY
import csv
rows = list(csv.DictReader(open("gpurun_out/${TAG}_prof/kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total ms", round(tot / 1e6, 2))
for r in rows[:14]:
    print(r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg", round(float(r["MinNs"]) / 1e3, 1), round(float(r["MaxNs"]) / 1e3, 1), r["Name"][:70])
PY
