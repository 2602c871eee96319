#!/bin/bash
# Spatial-sharding parity (tests/test_gpu_shard.py), then the N-rank rehearsal of bench.py's spatial leg.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/t_shard.log 2>&1 || { tail -60 gpurun_out/t_shard.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/t_shard.log | tail -8
bash tools/rehearse_ranks.sh 2 || { tail -30 gpurun_out/rehearse_2.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/rehearse_2.log") if l.startswith("{")][-1])
print("value", d["value"], "spatial", d["spatial"])
PY
