#!/bin/bash
# One GPU check on the current tree: -m gpu tests (optionally a subset: TESTS="tests/test_gpu_tsdf.py ..."), smoke(),
# and the default bench line.  Every step under its own time limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:?set TAG}
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 \
    || { echo SMOKE_FAILED; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
[ "${BENCH:-1}" = 1 ] || exit 0
timeout -k 10 400 python3 bench.py ${BENCH_ARGS} > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/${T}_bench.log; exit 1; }
tail -1 gpurun_out/${T}_bench.log > gpurun_out/${T}_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench.json'))
r=d['roofline']
print('value', d['value'], 'ms/step', d['ms_per_step'], 'kernel', r.get('kernel_ms_avg'), 'frac', r.get('frac'), 'eff', r.get('frac_effective'))
print('sustained', d.get('sustained'))
print('filtered', d['filtered']['ms_per_frame'], 'objects', d['objects']['ms'], d['objects']['single_object_ms'], d['objects']['objects_over_single'])"
