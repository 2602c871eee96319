#!/bin/bash
# configs[2] leg alone at several (batch, streams) settings: ms/frame per setting (bench.py's filtered object).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r02j}
for cfg in ${CFGS:-"32,1" "32,2" "32,3" "32,4" "16,4" "64,2"}; do
  b=${cfg%,*}; s=${cfg#*,}
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --cpu-frames 0 --sustain 0 --color64 0 --objects 0 \
      --hybrid-objects 0 --filter-frames ${FRAMES:-512} --filter-batch $b --filter-streams $s > gpurun_out/${TAG}_sweep_${b}_${s}.log 2>&1 || { echo "cfg $cfg failed"; tail -5 gpurun_out/${TAG}_sweep_${b}_${s}.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_sweep_${b}_${s}.log').read().strip().splitlines()[-1])['filtered'];print('batch $b streams $s', d['ms_per_frame'], d['mpoints_per_s'])"
done
