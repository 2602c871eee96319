#!/bin/bash
# Unprojection change check: filter / golden parity tests, then the configs[2] leg for the in-tree library and
# for variants/libotslam_<name>.so (A/B, alternating).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_filters.py tests/test_gpu_golden.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/unproj_tests.log 2>&1 || { tail -n 40 gpurun_out/unproj_tests.log; exit 1; }
tail -n 1 gpurun_out/unproj_tests.log
for name in base ${1:-old} base ${1:-old}; do
  lib=$PWD/object-triggered-3d-slam_amd/variants/libotslam_$name.so
  [ "$name" = base ] && lib=$PWD/object-triggered-3d-slam_amd/libotslam_hip.so
  OTSLAM_LIB=$lib timeout -k 10 300 python bench.py --frames 32 --steps 2 --cpu-frames 0 --objects 0 --hybrid-objects 0 > gpurun_out/b_unproj_$name.log 2>&1 || { tail -n 20 gpurun_out/b_unproj_$name.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/b_unproj_$name.log') if l.startswith('{')][-1]); f=d['filtered']; print('$name', f['mpoints_per_s'], f['ms_per_frame'])"
done
