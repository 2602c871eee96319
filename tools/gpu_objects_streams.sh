#!/bin/bash
# configs[3] with concurrent object streams: parity tests that touch the volume / mesh path, then the objects leg
# with 1 and 4 streams.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_tsdf.py tests/test_gpu_mesh.py tests/test_gpu_e2e.py \
    tests/test_gpu_shard.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_obj.log 2>&1 \
    || { tail -40 gpurun_out/t_obj.log; exit 1; }
tail -1 gpurun_out/t_obj.log
for T in 1 2 4; do
  timeout -k 10 300 python bench.py --frames 8 --steps 1 --cpu-frames 0 --filter-frames 0 --hybrid-objects 0 \
      --object-streams $T > gpurun_out/b_obj_$T.log 2>&1 || { tail -20 gpurun_out/b_obj_$T.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/b_obj_$T.log').read().splitlines()[-1]); o=d['objects']; print('streams $T', o['ms'], o['frames_per_s'], o['merged_points'])"
done
