#!/bin/bash
# One build-measure iteration on the GPU box: every -m gpu test, one object's kernel timeline (the timed fused path)
# and the default bench line.  TAG names the outputs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:?set TAG}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_obj_trace -o run -- python3 -u \
    tools/single_object_trace.py > gpurun_out/${T}_obj_trace.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/${T}_obj_trace.log; exit 1; }
python3 tools/single_object_trace.py --report gpurun_out/${T}_obj_trace/run_kernel_trace.csv > gpurun_out/${T}_obj_timeline.txt 2>&1
grep "host us per call of the timed\|single object" gpurun_out/${T}_obj_trace.log
grep span gpurun_out/${T}_obj_timeline.txt
timeout -k 10 400 python3 bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/${T}_bench.log; exit 1; }
tail -1 gpurun_out/${T}_bench.log > gpurun_out/${T}_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'kernel', d['roofline'].get('kernel_ms_avg'))
print('filtered', d['filtered']['ms_per_frame'], 'objects', d['objects']['ms'], d['objects']['single_object_ms'], d['objects']['objects_over_single'])"
echo DONE
