#!/bin/bash
# configs[2] iteration: batch-chain parity tests, then the per-frame time and rocprof breakdown (TAG = out prefix)
set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_filter_batch.py > gpurun_out/${TAG:-fb}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG:-fb}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG:-fb}_tests.log
bash tools/gpu_filter_prof.sh
