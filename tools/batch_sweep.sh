#!/bin/bash
# Time the headline TSDF step for several fused-batch sizes (frames per k_batch_integrate launch).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for b in ${BATCHES:-16 32 64}; do
  timeout -k 10 200 python bench.py --batch $b --steps 5 --cpu-frames 0 --filter-frames 0 --objects 0 \
      --hybrid-objects 0 > gpurun_out/bb_$b.log 2>&1 || exit 1
  python3 - "$b" <<'PY'
import json, sys
b = sys.argv[1]
d = json.loads(open(f"gpurun_out/bb_{b}.log").read().splitlines()[-1])
r = d["roofline"]
print(b, d["value"], d["ms_per_step"], r["kernel_ms_avg"], r["launches_per_step"])
PY
done
