#!/bin/bash
# configs[2] filter chain on the GPU box: parity tests (product library), per-frame timing of the product library and
# of the variants named in $VARIANTS (tools/variants.sh build), and a rocprofv3 kernel breakdown of the product run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r02f}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_filters.py tests/test_gpu_filter_batch.py tests/test_gpu_eval.py tests/test_gpu_sort.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_ftests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${TAG}_ftests.log; exit 1; }
tail -2 gpurun_out/${TAG}_ftests.log
fi
for v in base ${VARIANTS:-}; do
  timeout -k 10 300 python -u tools/with_variant.py $v tools/filter_batch_time.py --frames 64 --batches 32 > gpurun_out/${TAG}_fbt_$v.log 2>&1 || { tail -20 gpurun_out/${TAG}_fbt_$v.log; exit 1; }
  echo "$v: $(grep 'batch 32' gpurun_out/${TAG}_fbt_$v.log)"
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_fprof -o fb -- python3 tools/filter_batch_time.py --frames 64 --batches 32 --reps 2 > gpurun_out/${TAG}_fprof.log 2>&1 || { tail -20 gpurun_out/${TAG}_fprof.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/${TAG}_fprof gpurun_out/${TAG}_fprof/ks.csv | head -24
