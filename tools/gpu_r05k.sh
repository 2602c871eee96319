#!/bin/bash
# r05k: the sequence-tagged mailboxes (no events behind the units kernel / the marching-cubes scans) and the one-launch
# marching-cubes emission: mesh + TSDF parity, then one object's latency A/B (one launch vs the two-stream emission)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=r05k
timeout -k 10 600 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_tsdf.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for i in 1 2; do
  timeout -k 10 200 python3 -u tools/single_object_trace.py > gpurun_out/${T}_obj_${i}.log 2>&1 || { echo OBJ_FAILED; tail -20 gpurun_out/${T}_obj_${i}.log; exit 1; }
  grep "single object" gpurun_out/${T}_obj_${i}.log
  timeout -k 10 200 python3 -u tools/single_object_trace.py --fork > gpurun_out/${T}_objf_${i}.log 2>&1 || { echo OBJF_FAILED; tail -20 gpurun_out/${T}_objf_${i}.log; exit 1; }
  grep "single object" gpurun_out/${T}_objf_${i}.log
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_obj_trace -o run -- python3 -u \
    tools/single_object_trace.py > gpurun_out/${T}_obj_trace.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/${T}_obj_trace.log; exit 1; }
python3 tools/single_object_trace.py --report gpurun_out/${T}_obj_trace/run_kernel_trace.csv > gpurun_out/${T}_obj_timeline.txt 2>&1
head -30 gpurun_out/${T}_obj_timeline.txt
timeout -k 10 400 python3 bench.py --filter-frames 0 --hybrid-objects 0 --shard-steps 0 --sustain 0 > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/${T}_bench.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.log').read().strip().splitlines()[-1])
print('value', d['value'], 'objects', d['objects']['ms'], d['objects']['single_object_ms'], d['objects']['objects_over_single'])"
echo DONE
