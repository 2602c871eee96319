#!/bin/bash
# Rehearse bench.py's multi-rank path on a one-GPU box: N ranks share device 0, collectives over gloo.
# (The driver's scaling runs use RCCL with one GPU per rank; this checks sharding, merges and max-over-ranks timing.)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
N=${1:-2}
OT_BENCH_BACKEND=gloo OT_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus $N --steps 2 --warmup 1 --frames 64 --cpu-frames 0 \
  --filter-frames 0 > gpurun_out/rehearse_$N.log 2>&1
rc=$?
grep '^{' gpurun_out/rehearse_$N.log | tail -1
exit $rc
