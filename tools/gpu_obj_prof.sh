#!/bin/bash
# one configs[3] object's phases, then the same under rocprofv3 --kernel-trace (per-kernel breakdown; TAG = out dir)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-obj}
timeout -k 10 200 python3 -u tools/single_object_phases.py > gpurun_out/${TAG}_phases.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 -u tools/single_object_phases.py > gpurun_out/${TAG}_prof.log 2>&1
cat gpurun_out/${TAG}_phases.log
