#!/bin/bash
# configs[2] with concurrent frame streams: filter parity tests, then the leg with 1, 2 and 3 streams.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_filters.py tests/test_gpu_eval.py tests/test_gpu_change.py -m gpu \
    -x -q --timeout 200 --timeout-method thread > gpurun_out/t_filt.log 2>&1 || { tail -40 gpurun_out/t_filt.log; exit 1; }
tail -1 gpurun_out/t_filt.log
for T in ${STREAMS:-1 2 3}; do
  timeout -k 10 300 python bench.py --frames 8 --steps 1 --cpu-frames 0 --objects 0 --hybrid-objects 0 \
      --filter-frames 96 --filter-streams $T > gpurun_out/b_filt_$T.log 2>&1 || { tail -20 gpurun_out/b_filt_$T.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/b_filt_$T.log').read().splitlines()[-1]); f=d['filtered']; print('streams $T', f['ms_per_frame'], f['mpoints_per_s'], f['kept_per_frame'])"
done
