#!/bin/bash
# configs[2] batch chain alone, one stream: per-frame time + rocprofv3 kernel breakdown (TAG names the output dir)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-fb}
timeout -k 10 240 python3 -u tools/filter_batch_time.py --frames 64 --batches 32 --reps 3 > gpurun_out/${TAG}_time.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 -u tools/filter_batch_time.py --frames 64 --batches 32 --reps 3 > gpurun_out/${TAG}_prof.log 2>&1
cat gpurun_out/${TAG}_time.log
