#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 900 python -u -m pytest tests/test_gpu_filters.py tests/test_gpu_filter_batch.py tests/test_gpu_eval.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02a_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r02a_tests.log; exit 1; }
tail -3 gpurun_out/r02a_tests.log
timeout -k 10 300 python -u tools/filter_batch_time.py --frames 64 > gpurun_out/r02a_fbt.log 2>&1 || { tail -20 gpurun_out/r02a_fbt.log; exit 1; }
cat gpurun_out/r02a_fbt.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02a_prof -o fb -- python3 tools/filter_batch_time.py --frames 64 --batches 32 --reps 2 > gpurun_out/r02a_prof.log 2>&1 || { tail -20 gpurun_out/r02a_prof.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/r02a_prof gpurun_out/r02a_prof/ks.csv | head -30
