#!/bin/bash
# One GPU-box round trip: -m gpu tests (or $TESTS), the default bench line, and a rocprofv3 kernel-trace of the
# same bench command (summary -> gpurun_out/prof/kernel_stats.csv).  Stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TESTS=${TESTS:-tests}
BENCH_ARGS=${BENCH_ARGS:-}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py $BENCH_ARGS > gpurun_out/bench_prof.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/bench_prof.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof gpurun_out/prof/kernel_stats.csv
# headline leg alone: its k_batch_integrate average is the one bench.py's roofline reports (HIP events)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_h -o bench -- python3 bench.py \
    --objects 0 --hybrid-objects 0 --filter-frames 0 --cpu-frames 0 > gpurun_out/bench_prof_h.log 2>&1 || { echo PROF_H_FAILED; tail -30 gpurun_out/bench_prof_h.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_h gpurun_out/prof_h/kernel_stats.csv
tail -1 gpurun_out/bench_prof_h.log
echo DONE
