#!/bin/bash
# Rehearse the self-launched multi-rank bench on a one-GPU box: bench.py --gpus N (default 2) starts its own N ranks,
# all on device 0, collectives over gloo (no launcher).  TAG names the log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:?set TAG}
OT_BENCH_BACKEND=gloo OT_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 bench.py --gpus ${N:-2} --steps 5 --warmup 1 --cpu-frames 0 \
    --filter-frames 0 --sustain 0 --shard-steps 0 > gpurun_out/${T}_self${N:-2}.log 2>&1 || { echo SELF2_FAILED; tail -30 gpurun_out/${T}_self${N:-2}.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/${T}_self${N:-2}.log') if l.startswith('{')][-1])
print('n_gpus', d['n_gpus'], 'value', d['value'], 'objects', d['objects']['ms'], d['objects']['merge'][:60], 'spatial', (d.get('spatial') or {}).get('mesh_matches_unsharded'))"
echo DONE
