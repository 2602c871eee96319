#!/bin/bash
# Float64 chain parity (k_chain_*), mesh/sampling parity, then the configs[3] / configs[4] bench legs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_mesh.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > gpurun_out/t_chain.log 2>&1 || { tail -60 gpurun_out/t_chain.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/t_chain.log | tail -30
timeout -k 10 300 python bench.py --frames 8 --steps 1 --cpu-frames 0 --filter-frames 0 > gpurun_out/b_obj.log 2>&1 \
    || { tail -20 gpurun_out/b_obj.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/b_obj.log").read().splitlines()[-1])
print("objects", d["objects"])
print("hybrid", d["hybrid_map"])
PY
