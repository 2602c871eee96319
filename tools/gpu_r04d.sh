#!/bin/bash
# r04d: r04c plus a kernel timeline of one configs[3] object (tools/single_object_trace.py).
# isolated chain timing + rocprofv3 breakdown, then every -m gpu test and the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r04c}
timeout -k 10 600 python -u -m pytest tests/test_gpu_filter_batch.py tests/test_gpu_filters.py tests/test_gpu_chain.py tests/test_gpu_mesh.py tests/test_gpu_sort.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/${T}_filter_tests.log 2>&1 || { echo FILTER_TESTS_FAILED; tail -40 gpurun_out/${T}_filter_tests.log; exit 1; }
tail -1 gpurun_out/${T}_filter_tests.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 240 python3 -u tools/filter_batch_time.py --frames 64 --batches 32 --reps 3 > gpurun_out/${T}_fb_time.log 2>&1 || { echo FBTIME_FAILED; tail -20 gpurun_out/${T}_fb_time.log; exit 1; }
cat gpurun_out/${T}_fb_time.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_fb_prof -o run -- python3 -u tools/filter_batch_time.py --frames 64 --batches 32 --reps 3 > gpurun_out/${T}_fb_prof.log 2>&1 || { echo FBPROF_FAILED; tail -20 gpurun_out/${T}_fb_prof.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_filter_batch.py --deselect tests/test_gpu_filters.py --deselect tests/test_gpu_chain.py --deselect tests/test_gpu_mesh.py --deselect tests/test_gpu_sort.py > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/${T}_bench.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.log').read().strip().splitlines()[-1])
print('value', d['value'], 'filtered', d['filtered']['ms_per_frame'], 'objects', d['objects']['ms'], d['objects']['single_object_ms'], d['objects']['objects_over_single'])
print('amdahl', d['spatial_amdahl'])"
timeout -k 10 200 python3 tools/single_object_phases.py > gpurun_out/${T}_obj_phases.log 2>&1 || { echo PHASES_FAILED; tail -20 gpurun_out/${T}_obj_phases.log; exit 1; }
cat gpurun_out/${T}_obj_phases.log

cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_obj_trace -o run -- python3 -u tools/single_object_trace.py > gpurun_out/${T}_obj_trace.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/${T}_obj_trace.log; exit 1; }
python3 tools/single_object_trace.py --report gpurun_out/${T}_obj_trace/run_kernel_trace.csv > gpurun_out/${T}_obj_timeline.txt 2>&1
grep -E "single object|units|priority" gpurun_out/${T}_obj_trace.log || true
tail -30 gpurun_out/${T}_obj_timeline.txt
echo DONE
