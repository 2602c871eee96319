#!/bin/bash
# Marching-cubes iteration: mesh / configs / shard parity, then one object's timeline (TAG names the outputs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:?set TAG}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_configs_full.py tests/test_gpu_shard.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_obj_trace -o run -- python3 -u \
    tools/single_object_trace.py > gpurun_out/${T}_obj_trace.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/${T}_obj_trace.log; exit 1; }
python3 tools/single_object_trace.py --report gpurun_out/${T}_obj_trace/run_kernel_trace.csv > gpurun_out/${T}_obj_timeline.txt 2>&1
grep "single object" gpurun_out/${T}_obj_trace.log
grep -E "k_mc_|span" gpurun_out/${T}_obj_timeline.txt | head -9
for i in 1 2 3; do
  timeout -k 10 200 python3 -u tools/single_object_trace.py > gpurun_out/${T}_obj.log 2>&1 || { echo OBJ_FAILED; exit 1; }
  grep "single object" gpurun_out/${T}_obj.log
done
echo DONE
