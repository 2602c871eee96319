#!/bin/bash
# TSDF parity (incl. the full-size bench workload) and the headline bench line, TSDF leg only.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 500 python -u -m pytest tests/test_gpu_tsdf.py tests/test_gpu_bench_scale.py tests/test_gpu_mesh.py \
    tests/test_gpu_e2e.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_tsdf.log 2>&1 \
    || { tail -40 gpurun_out/t_tsdf.log; exit 1; }
tail -2 gpurun_out/t_tsdf.log
BATCHES=32 bash tools/batch_sweep.sh
