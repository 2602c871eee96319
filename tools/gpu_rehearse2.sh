#!/bin/bash
# The N=2 bench path rehearsed on the one-GPU box: two ranks on device 0, collectives over gloo (host memory).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r02u}
OT_BENCH_BACKEND=gloo OT_BENCH_SHARE_GPU=1 timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps ${STEPS:-10} --warmup 2 --cpu-frames 0 \
    --sustain 0 --color64 0 --filter-frames 64 > gpurun_out/${TAG}_rehearse2.log 2>&1 || { echo REHEARSE_FAILED; tail -30 gpurun_out/${TAG}_rehearse2.log; exit 1; }
grep '^{' gpurun_out/${TAG}_rehearse2.log | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(json.dumps({k:d[k] for k in ('value','n_gpus','spatial','objects')})[:1500])"
