#!/bin/bash
# One object's kernels against the host's launch calls (kernel + HIP runtime API trace, no counters).  TAG names outputs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:?set TAG}
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/${T}_lag -o run -- \
    python3 -u tools/single_object_trace.py > gpurun_out/${T}_lag.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/${T}_lag.log; exit 1; }
ls gpurun_out/${T}_lag
python3 tools/launch_lag.py gpurun_out/${T}_lag/run_kernel_trace.csv gpurun_out/${T}_lag/run_hip_api_trace.csv \
    > gpurun_out/${T}_lag.txt 2>&1; cat gpurun_out/${T}_lag.txt
echo DONE
