#!/bin/bash
# One GPU-box round trip: -m gpu tests (or $TESTS), the default bench line, a rocprofv3 kernel-trace of the same
# bench command and of the headline leg alone; PMC=1 first runs the PMC passes that produce profiles/pmc_traffic.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TESTS=${TESTS:-tests}
BENCH_ARGS=${BENCH_ARGS:-}
TAG=${TAG:-r02}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_gpu_tests.log
fi
if [ "${PMC:-0}" = 1 ]; then  # first, so that the bench line below reads the same-hash counter traffic
bash tools/pmc.sh || exit 1
fi
timeout -k 10 400 python bench.py $BENCH_ARGS > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
if [ "${PROF:-1}" = 1 ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o bench -- python3 bench.py $BENCH_ARGS > gpurun_out/${TAG}_bench_prof.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/${TAG}_bench_prof.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/${TAG}_prof gpurun_out/${TAG}_prof/kernel_stats.csv > /dev/null
# headline leg alone: its k_batch_integrate average is the one bench.py's roofline reports (HIP events)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_h -o bench -- python3 bench.py \
    --objects 0 --hybrid-objects 0 --filter-frames 0 --cpu-frames 0 --sustain 0 > gpurun_out/${TAG}_bench_prof_h.log 2>&1 || { echo PROF_H_FAILED; tail -30 gpurun_out/${TAG}_bench_prof_h.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/${TAG}_prof_h gpurun_out/${TAG}_prof_h/kernel_stats.csv > /dev/null
grep -h "k_batch_integrate" gpurun_out/${TAG}_prof_h/kernel_stats.csv | cut -c1-120
fi
echo DONE
