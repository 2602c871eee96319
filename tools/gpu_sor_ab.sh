#!/bin/bash
# A/B of a SOR test hook on one GPU box: the SOR / filter-chain parity tests, then the configs[2] chain under
# rocprofv3 --kernel-trace --stats with the hook alternating 1 / 0 in one process (the two template variants show up
# as separate kernels).  TAG names the outputs; HOOK (default otx_sor_netfill), ROUNDS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:?set TAG}
HOOK=${HOOK:-otx_sor_netfill}
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_filters.py tests/test_gpu_filter_batch.py} -m gpu -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
[ "${SKIP_TESTS:-0}" = 1 ] || tail -1 gpurun_out/${TAG}_tests.log
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o fb -- python3 -u tools/filter_batch_time.py \
    --frames 64 --batches 64 --reps 2 --ab-netfill ${ROUNDS:-3} --ab-hook $HOOK > gpurun_out/${TAG}_fbt.log 2>&1 \
    || { echo PROF_FAILED; tail -20 gpurun_out/${TAG}_fbt.log; exit 1; }
grep -E "batch 64|$HOOK" gpurun_out/${TAG}_fbt.log
python3 tools/prof_summary.py gpurun_out/${TAG}_prof gpurun_out/${TAG}_prof/kernel_stats.csv > /dev/null
python3 - <<PY
import csv
rows = list(csv.DictReader(open("gpurun_out/${TAG}_prof/kernel_stats.csv")))
for r in rows:
    if "sor" in r["Name"] or rows.index(r) < 6:
        print(r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg", round(float(r["MinNs"]) / 1e3, 1),
              round(float(r["MaxNs"]) / 1e3, 1), r["Name"][:90])
PY
echo DONE
