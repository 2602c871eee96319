#!/bin/bash
# Sharding iteration on the GPU box: the shard / TSDF parity tests, then tools/shard_scaling.py (every rank's step,
# front end and integrate per batch; ownership blocks vs sectors, fused vs split front end).  TAG names the outputs;
# SCALE_ARGS are passed to the tool.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:?set TAG}
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_shard.py tests/test_gpu_tsdf.py} -m gpu -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/${T}_gpu_tests.log; exit 1; }
[ "${SKIP_TESTS:-0}" = 1 ] || tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 600 python3 -u tools/shard_scaling.py ${SCALE_ARGS} > gpurun_out/${T}_scaling.log 2>&1 \
    || { echo SCALING_FAILED; tail -30 gpurun_out/${T}_scaling.log; exit 1; }
grep "^N " gpurun_out/${T}_scaling.log
echo DONE
