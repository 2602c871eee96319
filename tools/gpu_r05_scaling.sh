#!/bin/bash
# TSDF / shard parity tests, then tools/shard_scaling.py (rank 0's shard integrate + front end per batch for 1..64 ranks)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
T=${TAG:?set TAG}
timeout -k 10 600 python -u -m pytest tests/test_gpu_tsdf.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 300 python3 -u tools/shard_scaling.py > gpurun_out/${T}_scaling.log 2>&1 || { echo SCALING_FAILED; tail -20 gpurun_out/${T}_scaling.log; exit 1; }
grep "^N" gpurun_out/${T}_scaling.log
