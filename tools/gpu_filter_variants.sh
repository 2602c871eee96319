#!/bin/bash
# configs[2] A/B: the batch-chain parity tests on the product library, then per variant (base = product) the per-frame
# time and a rocprofv3 kernel breakdown of the same run (tools/prof_table.py reads gpurun_out/fbv_<name>_prof)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_filter_batch.py > gpurun_out/fbv_tests.log 2>&1 || { tail -30 gpurun_out/fbv_tests.log; exit 1; }
tail -1 gpurun_out/fbv_tests.log
for name in "$@"; do
  timeout -k 10 200 python3 -u tools/with_variant.py $name tools/filter_batch_time.py --frames 64 --batches 32 --reps 5 > gpurun_out/fbv_${name}_time.log 2>&1
  echo "$name $(grep batch gpurun_out/fbv_${name}_time.log)"
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/fbv_${name}_prof -o run -- python3 -u tools/with_variant.py $name tools/filter_batch_time.py --frames 64 --batches 32 --reps 3 > gpurun_out/fbv_${name}_prof.log 2>&1
done
