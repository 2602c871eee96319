#!/bin/bash
# round-3 check: full -m gpu suite, default bench line, kernel variants A/B, single-object phases + kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r03b}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-1500
bash tools/gpu_ab_bench.sh ${VARIANTS:-base} || exit 1
timeout -k 10 200 python3 tools/single_object_phases.py > gpurun_out/${TAG}_phases.log 2>&1 || { echo PHASES_FAILED; tail -20 gpurun_out/${TAG}_phases.log; exit 1; }
cat gpurun_out/${TAG}_phases.log | tail -12
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_obj -o obj -- python3 tools/single_object_phases.py > gpurun_out/${TAG}_prof_obj.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/${TAG}_prof_obj.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/${TAG}_prof_obj gpurun_out/${TAG}_prof_obj/kernel_stats.csv > /dev/null
head -25 gpurun_out/${TAG}_prof_obj/kernel_stats.csv | cut -c1-160
echo DONE
