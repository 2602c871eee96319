#!/bin/bash
# Marching-cubes change check: mesh / e2e / golden / shard parity tests, then the configs[3] objects leg under
# rocprofv3 kernel-trace (summary -> gpurun_out/prof_obj/kernel_stats.csv).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_mesh.py tests/test_gpu_e2e.py tests/test_gpu_golden.py tests/test_gpu_shard.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mc_tests.log 2>&1 || { echo TESTS_FAILED; tail -n 40 gpurun_out/mc_tests.log; exit 1; }
tail -n 2 gpurun_out/mc_tests.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_obj -o bench -- python3 bench.py \
    --hybrid-objects 0 --filter-frames 0 --cpu-frames 0 > gpurun_out/bench_obj.log 2>&1 || { echo PROF_FAILED; tail -n 30 gpurun_out/bench_obj.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_obj gpurun_out/prof_obj/kernel_stats.csv
python3 -c "import json;d=json.loads([l for l in open('gpurun_out/bench_obj.log') if l.startswith('{')][-1]);print(d['value'], d['objects'])"
grep -E "k_mc|k_batch_integrate" gpurun_out/prof_obj/kernel_stats.csv | cut -d, -f1-4
