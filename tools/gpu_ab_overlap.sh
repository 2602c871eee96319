#!/bin/bash
# headline with / without the double-buffered front end (A, B, A) and the per-rank sharded steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
A="--filter-frames 0 --objects 0 --hybrid-objects 0 --cpu-frames 0 --sustain 0 --color32 0 --steps 100"
timeout -k 10 300 python3 bench.py $A > gpurun_out/${TAG:-r05b}_def.log 2>&1 || { echo FAIL1; tail -20 gpurun_out/${TAG:-r05b}_def.log; exit 1; }
timeout -k 10 300 python3 bench.py $A --overlap 1 --shard-steps 0 > gpurun_out/${TAG:-r05b}_ovl.log 2>&1 || { echo FAIL2; tail -20 gpurun_out/${TAG:-r05b}_ovl.log; exit 1; }
timeout -k 10 300 python3 bench.py $A --shard-steps 0 > gpurun_out/${TAG:-r05b}_def2.log 2>&1 || { echo FAIL3; tail -20 gpurun_out/${TAG:-r05b}_def2.log; exit 1; }
TAG=${TAG:-r05b} python3 - <<'PY'
import json, os
tag = os.environ["TAG"]
for t in ("def", "ovl", "def2"):
    d = json.loads(open(f"gpurun_out/{tag}_{t}.log").read().strip().splitlines()[-1])
    print(t, d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_avg"])
d = json.loads(open(f"gpurun_out/{tag}_def.log").read().strip().splitlines()[-1])
print(json.dumps(d["spatial_amdahl"]["measured"]["worlds"]))
PY
