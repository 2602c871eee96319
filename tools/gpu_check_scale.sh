#!/bin/bash
# Full-size configs[1] parity test, then the fused-batch-size sweep (tools/batch_sweep.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_scale.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/t_bs.log 2>&1 || { tail -30 gpurun_out/t_bs.log; exit 1; }
tail -2 gpurun_out/t_bs.log
bash tools/batch_sweep.sh
