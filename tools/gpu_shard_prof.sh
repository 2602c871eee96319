#!/bin/bash
# Kernel timelines of one rank's shard (tools/shard_trace.py under rocprofv3 --kernel-trace): TRACES is a list of
# "name:args" (args passed to shard_trace.py); then an optional tools/shard_scaling.py run (SCALE_ARGS).  TAG names the
# outputs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:?set TAG}
for tr in ${TRACES}; do
  n=${tr%%:*}; args=${tr#*:}; args=${args//,/ }
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_${n} -o run -- python3 -u \
      tools/shard_trace.py ${args} > gpurun_out/${T}_${n}.log 2>&1 || { echo TRACE_FAILED $n; tail -20 gpurun_out/${T}_${n}.log; exit 1; }
  grep "ms/step" gpurun_out/${T}_${n}.log
  python3 tools/shard_trace.py --report gpurun_out/${T}_${n}/run_kernel_trace.csv > gpurun_out/${T}_${n}_timeline.txt 2>&1
  grep -A12 "^span" gpurun_out/${T}_${n}_timeline.txt
done
if [ -n "${SCALE_ARGS}" ]; then
  timeout -k 10 600 python3 -u tools/shard_scaling.py ${SCALE_ARGS} > gpurun_out/${T}_scaling.log 2>&1 \
      || { echo SCALING_FAILED; tail -30 gpurun_out/${T}_scaling.log; exit 1; }
  grep "^N " gpurun_out/${T}_scaling.log
fi
echo DONE
