#!/bin/bash
# r05m: the timed (fused) single-object sequence: kernel timelines with the normals starting after the emission (0) or
# beside the area-sum walk (1), and the host's share of the wall time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=r05m
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
for a in 0 1; do
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_obj_trace${a} -o run -- python3 -u \
    tools/single_object_trace.py --normals-at $a > gpurun_out/${T}_obj_trace${a}.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/${T}_obj_trace${a}.log; exit 1; }
python3 tools/single_object_trace.py --report gpurun_out/${T}_obj_trace${a}/run_kernel_trace.csv > gpurun_out/${T}_obj_timeline${a}.txt 2>&1
grep "host us\|single object" gpurun_out/${T}_obj_trace${a}.log
grep "span" gpurun_out/${T}_obj_timeline${a}.txt
done
for a in 0 1 2; do
timeout -k 10 200 python3 -u tools/single_object_trace.py --normals-at $a > gpurun_out/${T}_obj_${a}.log 2>&1 || { echo OBJ_FAILED; exit 1; }
grep "host us per call of the timed\|single object" gpurun_out/${T}_obj_${a}.log
done
echo DONE
