#!/bin/bash
# r04aa: single-object latency work (one-launch unit sort, sampler tables carried by the areas launch, mailed totals):
# the affected -m gpu tests, one object's kernel timeline, the same object without normals, then the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r04aa}
timeout -k 10 600 python -u -m pytest tests/test_gpu_tsdf.py tests/test_gpu_mesh.py tests/test_gpu_chain.py tests/test_gpu_sort.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 300 python3 -u tools/chain_walk_trace.py > gpurun_out/${T}_walk_trace.log 2>&1 || { echo WALK_TRACE_FAILED; tail -20 gpurun_out/${T}_walk_trace.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_walk_trace.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_obj_trace -o run -- python3 -u tools/single_object_trace.py > gpurun_out/${T}_obj_trace.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/${T}_obj_trace.log; exit 1; }
python3 tools/single_object_trace.py --report gpurun_out/${T}_obj_trace/run_kernel_trace.csv > gpurun_out/${T}_obj_timeline.txt 2>&1
grep -E "single object|units" gpurun_out/${T}_obj_trace.log || true
timeout -k 10 200 python3 -u tools/single_object_trace.py > gpurun_out/${T}_obj_plain.log 2>&1 || { echo PLAIN_FAILED; tail -20 gpurun_out/${T}_obj_plain.log; exit 1; }
grep -E "single object|host us" gpurun_out/${T}_obj_plain.log
timeout -k 10 200 python3 -u tools/single_object_trace.py --no-normals > gpurun_out/${T}_obj_nonormals.log 2>&1 || { echo NONORMALS_FAILED; tail -20 gpurun_out/${T}_obj_nonormals.log; exit 1; }
grep -E "single object|host us" gpurun_out/${T}_obj_nonormals.log
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/${T}_bench.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.log').read().strip().splitlines()[-1])
print('value', d['value'], 'filtered', d['filtered']['ms_per_frame'], 'objects', d['objects']['ms'], d['objects']['single_object_ms'], d['objects']['objects_over_single'])"
head -45 gpurun_out/${T}_obj_timeline.txt
echo DONE
