#!/bin/bash
# r04b: the RAW (unstaged) sharded integrate: shard parity tests, then one rank's kernels alone on the GPU at world
# 1 / 2 / 4 / 8 under rocprofv3 (tools/shard_frontend.py), and the single-object phase profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r04b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_tsdf.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/${T}_shard_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_shard_tests.log; exit 1; }
tail -1 gpurun_out/${T}_shard_tests.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
for w in 1 2 4 8; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_shard_w$w -o run -- \
    python3 tools/shard_frontend.py --world $w --reps 20 > gpurun_out/${T}_shard_w$w.log 2>&1 || { echo SHARD_$w FAILED; tail -20 gpurun_out/${T}_shard_w$w.log; exit 1; }
  grep world gpurun_out/${T}_shard_w$w.log
done
timeout -k 10 200 python3 tools/single_object_phases.py > gpurun_out/${T}_obj_phases.log 2>&1 || { echo PHASES_FAILED; tail -20 gpurun_out/${T}_obj_phases.log; exit 1; }
cat gpurun_out/${T}_obj_phases.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_obj -o run -- \
  python3 tools/single_object_phases.py > gpurun_out/${T}_obj_prof.log 2>&1 || { echo OBJPROF_FAILED; tail -20 gpurun_out/${T}_obj_prof.log; exit 1; }
echo DONE
