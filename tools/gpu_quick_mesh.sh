#!/bin/bash
# quick check: the mesh / marching-cubes GPU tests, then one object's timing with and without normals
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-quick}
timeout -k 10 400 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_tsdf.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 200 python3 -u tools/single_object_trace.py > gpurun_out/${T}_obj_plain.log 2>&1 || { echo PLAIN_FAILED; tail -20 gpurun_out/${T}_obj_plain.log; exit 1; }
grep -E "single object|host us" gpurun_out/${T}_obj_plain.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_obj_trace -o run -- python3 -u tools/single_object_trace.py > gpurun_out/${T}_obj_trace.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/${T}_obj_trace.log; exit 1; }
python3 tools/single_object_trace.py --report gpurun_out/${T}_obj_trace/run_kernel_trace.csv > gpurun_out/${T}_obj_timeline.txt 2>&1
grep -E "vnormals|walk|bsum|guess|span" gpurun_out/${T}_obj_timeline.txt | head -12
echo DONE
