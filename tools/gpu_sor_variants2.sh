#!/bin/bash
# SOR variant A/B on one GPU box: per variant (tools/variants.sh build) the SOR / filter-chain parity tests against
# that library, then the configs[2] batch timing under rocprofv3 (kernel breakdown per variant).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
for v in ${VARIANTS:-base}; do
  timeout -k 10 300 python -u tools/with_variant.py $v -m pytest tests/test_gpu_filters.py tests/test_gpu_filter_batch.py -m gpu -x -q -k "sor or batch" --timeout 120 --timeout-method thread > gpurun_out/sv_${v}_tests.log 2>&1 || { echo "$v TESTS_FAILED"; tail -30 gpurun_out/sv_${v}_tests.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/sv_${v}_tests.log)"
  cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sv_${v}_prof -o fb -- python3 tools/with_variant.py $v tools/filter_batch_time.py --frames 64 --batches 32 > gpurun_out/sv_${v}_fbt.log 2>&1 || { echo "$v PROF_FAILED"; tail -20 gpurun_out/sv_${v}_fbt.log; exit 1; }
  echo "$v $(grep 'batch 32' gpurun_out/sv_${v}_fbt.log)"
  python3 tools/prof_summary.py gpurun_out/sv_${v}_prof gpurun_out/sv_${v}_prof/kernel_stats.csv > /dev/null
  python3 - <<PY
import csv
rows = list(csv.DictReader(open("gpurun_out/sv_${v}_prof/kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("  total ms", round(tot / 1e6, 2))
for r in rows:
    if "sor" in r["Name"] or "cell_nbr" in r["Name"] or "fb_reduce" in r["Name"]:
        print("  ", r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg", r["Name"][:50])
PY
done
