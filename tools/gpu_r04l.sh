#!/bin/bash
# r04l: chain-walk event trace of a configs[3] mesh (where the sampling chains' walk time goes), then the r04d set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r04l}
timeout -k 10 300 python3 -u tools/chain_walk_trace.py > gpurun_out/${T}_walk_trace.log 2>&1 || { echo WALK_TRACE_FAILED; tail -20 gpurun_out/${T}_walk_trace.log; exit 1; }
cat gpurun_out/${T}_walk_trace.log
TAG=$T bash tools/gpu_r04d.sh
