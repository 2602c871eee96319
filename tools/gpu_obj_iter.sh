#!/bin/bash
# One-object latency iteration: the mesh / configs[3] / shard parity tests (TESTS overrides), then one object's kernel
# timeline (tools/single_object_trace.py under rocprofv3 --kernel-trace).  TAG names the outputs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:?set TAG}
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_mesh.py tests/test_gpu_configs_full.py tests/test_gpu_e2e.py tests/test_gpu_golden.py tests/test_gpu_shard.py} \
    -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 \
    || { echo TESTS_FAILED; tail -60 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_obj_trace -o run -- python3 -u \
    tools/single_object_trace.py > gpurun_out/${T}_obj_trace.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/${T}_obj_trace.log; exit 1; }
python3 tools/single_object_trace.py --report gpurun_out/${T}_obj_trace/run_kernel_trace.csv > gpurun_out/${T}_obj_timeline.txt 2>&1
grep -E "single object|host us" gpurun_out/${T}_obj_trace.log
grep -E "span|k_mc_|k_batch_integrate" gpurun_out/${T}_obj_timeline.txt | tail -12
echo DONE
