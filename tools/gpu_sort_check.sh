#!/bin/bash
# Radix sort parity, then every GPU test (the sort orders units, edges, voxels and grids), then the filter leg.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/t_sort.log 2>&1 || { tail -40 gpurun_out/t_sort.log; exit 1; }
tail -1 gpurun_out/t_sort.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/t_all.log 2>&1 || { tail -40 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 300 python bench.py --frames 8 --steps 1 --cpu-frames 0 > gpurun_out/b_sort.log 2>&1 \
    || { tail -20 gpurun_out/b_sort.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/b_sort.log').read().splitlines()[-1]); print('filtered', d['filtered']['ms_per_frame'], 'objects', d['objects']['ms'], 'hybrid', d['hybrid_map']['ms'])"
