#!/bin/bash
# SOR grid-shape variants: parity (HD batch + SOR tests) then the batched configs[2] chain timing, per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in ${VARIANTS:-base}; do
  timeout -k 10 400 python -u tools/with_variant.py $v -m pytest tests/test_gpu_filter_batch.py tests/test_gpu_filters.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hd_batch or sor or wide or ragged" > gpurun_out/sv_test_$v.log 2>&1 || { echo "$v TESTS FAILED"; tail -30 gpurun_out/sv_test_$v.log; exit 1; }
  timeout -k 10 300 python -u tools/with_variant.py $v tools/filter_batch_time.py --frames 128 --batches 32,64 > gpurun_out/sv_time_$v.log 2>&1 || { echo "$v TIME FAILED"; tail -20 gpurun_out/sv_time_$v.log; exit 1; }
  echo "== $v: $(tail -1 gpurun_out/sv_test_$v.log)"; grep batch gpurun_out/sv_time_$v.log
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in ${PROF:-base}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sv_prof_$v -o fb -- python3 tools/with_variant.py $v tools/filter_batch_time.py --frames 64 --batches 32 --reps 2 > gpurun_out/sv_prof_$v.log 2>&1 || { tail -20 gpurun_out/sv_prof_$v.log; exit 1; }
  python3 tools/prof_summary.py gpurun_out/sv_prof_$v gpurun_out/sv_prof_$v/ks.csv > /dev/null
  echo "== prof $v"; cut -c1-150 gpurun_out/sv_prof_$v/ks.csv | head -14
done
