#!/bin/bash
# A/B on one GPU box: the filter-chain parity tests + TSDF tests on the product library, then filter_batch timing and
# the bench line for the product library ("base") and each variant in $VARIANTS (tools/variants.sh / with_variant.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-ab}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_filter_batch.py tests/test_gpu_tsdf.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for v in base ${VARIANTS:-} base ${VARIANTS:-}; do
  timeout -k 10 300 python -u tools/with_variant.py $v tools/filter_batch_time.py --frames 64 --batches 32 > gpurun_out/${TAG}_fbt_$v.log 2>&1 || { tail -20 gpurun_out/${TAG}_fbt_$v.log; exit 1; }
  echo "$v filter: $(grep 'batch 32' gpurun_out/${TAG}_fbt_$v.log)"
  timeout -k 10 300 python -u tools/with_variant.py $v bench.py --cpu-frames 0 ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench_$v.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_$v.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_bench_$v.log').read().strip().splitlines()[-1]);print('$v bench', d['value'], 'c64', d['color64']['frames_per_s'], d['color64']['kernel_ms_avg'], 'filt ms/frame', d['filtered']['ms_per_frame'])"
done
