#!/bin/bash
# r05l: where the fused extraction lets the vertex normals start (after the emission / beside the sum walk / beside the
# CDF walk), with mesh parity first; event / kernel-argument gap microbenchmark
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=r05l
timeout -k 10 60 ./tools/event_gap 300 > gpurun_out/${T}_event_gap.log 2>&1 && cat gpurun_out/${T}_event_gap.log || { echo GAP_FAILED; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_mesh.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for i in 1 2; do
  for a in 0 1 2; do
    timeout -k 10 200 python3 -u tools/single_object_trace.py --normals-at $a > gpurun_out/${T}_obj_${a}_${i}.log 2>&1 || { echo OBJ_FAILED; tail -20 gpurun_out/${T}_obj_${a}_${i}.log; exit 1; }
    grep "single object" gpurun_out/${T}_obj_${a}_${i}.log
  done
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
for a in 1 2; do
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_obj_trace${a} -o run -- python3 -u \
    tools/single_object_trace.py --normals-at $a > gpurun_out/${T}_obj_trace${a}.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/${T}_obj_trace${a}.log; exit 1; }
python3 tools/single_object_trace.py --report gpurun_out/${T}_obj_trace${a}/run_kernel_trace.csv > gpurun_out/${T}_obj_timeline${a}.txt 2>&1
done
timeout -k 10 400 python3 bench.py --filter-frames 0 --hybrid-objects 0 --shard-steps 0 --sustain 0 > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/${T}_bench.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.log').read().strip().splitlines()[-1])
print('value', d['value'], 'objects', d['objects']['ms'], d['objects']['single_object_ms'], d['objects']['objects_over_single'])"
echo DONE
