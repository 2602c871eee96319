#!/bin/bash
# SOR cell-occupancy sweep (OT_SOR_OCC = target points per occupied cell) on the configs[2] leg, one stream.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for occ in ${OCCS:-8 10 12 14 17 20}; do
  OT_SOR_OCC=$occ timeout -k 10 200 python bench.py --frames 8 --steps 1 --cpu-frames 0 --objects 0 --hybrid-objects 0 \
      --filter-frames 96 --filter-streams 1 > gpurun_out/sweep_$occ.log 2>&1 || { tail -5 gpurun_out/sweep_$occ.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/sweep_$occ.log').read().splitlines()[-1]);print($occ, d['filtered']['ms_per_frame'], d['filtered']['kept_per_frame'])"
done
