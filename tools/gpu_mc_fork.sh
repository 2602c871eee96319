#!/bin/bash
# One object's timeline with the marching-cubes emission as two kernels on two streams (times each half)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:?set TAG}
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_fork_trace -o run -- python3 -u \
    tools/single_object_trace.py --fork > gpurun_out/${T}_fork_trace.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/${T}_fork_trace.log; exit 1; }
python3 tools/single_object_trace.py --report gpurun_out/${T}_fork_trace/run_kernel_trace.csv > gpurun_out/${T}_fork_timeline.txt 2>&1
grep -E "k_mc_|span" gpurun_out/${T}_fork_timeline.txt | head -9
echo DONE
