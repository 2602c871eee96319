#!/bin/bash
# Change-detection parity (incl. the multi-object voxel-key diff) and the configs[3] / configs[4] bench legs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_change.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > gpurun_out/t_chg.log 2>&1 || { tail -40 gpurun_out/t_chg.log; exit 1; }
tail -12 gpurun_out/t_chg.log
timeout -k 10 300 python bench.py --frames 8 --steps 1 --cpu-frames 0 --filter-frames 0 > gpurun_out/b_obj.log 2>&1 \
    || { tail -20 gpurun_out/b_obj.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/b_obj.log").read().splitlines()[-1])
print("objects", d["objects"])
print("hybrid", d["hybrid_map"])
PY
