#!/bin/bash
# Filter parity (unproject / voxel / SOR / ROR / NN incl. the configs[2] frame), then the configs[2] bench leg.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_filters.py tests/test_gpu_eval.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/t_filt.log 2>&1 || { tail -40 gpurun_out/t_filt.log; exit 1; }
tail -1 gpurun_out/t_filt.log
timeout -k 10 300 python bench.py --frames 8 --steps 1 --cpu-frames 0 --objects 0 --hybrid-objects 0 \
    --filter-frames 64 > gpurun_out/b_filt.log 2>&1 || { tail -20 gpurun_out/b_filt.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/b_filt.log').read().splitlines()[-1]); print(d['filtered'])"
