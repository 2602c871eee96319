#!/bin/bash
# Round records on the final build (part A): every -m gpu test, smoke(), the default bench line, the rocprofv3
# headline kernel stats (the roofline's kernel time cross-check), the configs[2] kernel breakdown and one object's
# kernel timeline.  Part B is tools/pmc.sh (same-hash PMC traffic for the bench's roofline objects).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:?set TAG, e.g. r05z}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 \
    || { echo SMOKE_FAILED; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/${T}_bench.log; exit 1; }
tail -1 gpurun_out/${T}_bench.log > gpurun_out/${T}_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'roofline', d['roofline'].get('frac'), d['roofline'].get('kernel_ms_avg'))
print('filtered', d['filtered']['ms_per_frame'], 'objects', d['objects']['ms'], d['objects']['single_object_ms'], d['objects']['objects_over_single'])"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_h -o bench -- python3 bench.py \
    --objects 0 --hybrid-objects 0 --filter-frames 0 --cpu-frames 0 --sustain 0 --shard-steps 0 --color32 0 \
    > gpurun_out/${T}_bench_prof_h.log 2>&1 \
    || { echo PROF_FAILED; tail -30 gpurun_out/${T}_bench_prof_h.log; exit 1; }
tail -1 gpurun_out/${T}_bench_prof_h.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_fb_prof -o run -- python3 -u \
    tools/filter_batch_time.py --frames 128 --batches 64 --reps 3 > gpurun_out/${T}_fb_prof.log 2>&1 \
    || { echo FBPROF_FAILED; tail -20 gpurun_out/${T}_fb_prof.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_obj_trace -o run -- python3 -u \
    tools/single_object_trace.py > gpurun_out/${T}_obj_trace.log 2>&1 || { echo TRACE_FAILED; tail -20 gpurun_out/${T}_obj_trace.log; exit 1; }
python3 tools/single_object_trace.py --report gpurun_out/${T}_obj_trace/run_kernel_trace.csv > gpurun_out/${T}_obj_timeline.txt 2>&1
grep -E "single object|units" gpurun_out/${T}_obj_trace.log || true
grep -E "k_batch_integrate|k_sor_knn<" gpurun_out/${T}_prof_h/*stats.csv gpurun_out/${T}_fb_prof/*stats.csv | cut -c1-200 || true
echo DONE
