#!/bin/bash
# Round-5 A/B on one box: filter parity tests, the SOR stage-1 network fill (alternating in one process), the headline
# with and without the double-buffered front end, and the per-rank sharded steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
T=${TAG:?set TAG}
timeout -k 10 600 python -u -m pytest tests/test_gpu_filters.py tests/test_gpu_filter_batch.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/${T}_ftests.log 2>&1 || { echo FTESTS_FAILED; tail -40 gpurun_out/${T}_ftests.log; exit 1; }
tail -1 gpurun_out/${T}_ftests.log
timeout -k 10 400 python3 -u tools/filter_batch_time.py --frames 128 --batches 64 --reps 1 --ab-netfill 3 \
    > gpurun_out/${T}_netfill.log 2>&1 || { echo NETFILL_FAILED; tail -20 gpurun_out/${T}_netfill.log; exit 1; }
grep -E "netfill|batch 64" gpurun_out/${T}_netfill.log
bash tools/gpu_ab_overlap.sh
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
for ov in 1 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_shard8_ov$ov -o run -- python3 -u \
      tools/shard_trace.py --world 8 --overlap $ov > gpurun_out/${T}_shard8_ov$ov.log 2>&1 || { echo SHARDTRACE_FAILED; tail -20 gpurun_out/${T}_shard8_ov$ov.log; exit 1; }
  grep "ms/step" gpurun_out/${T}_shard8_ov$ov.log
  python3 tools/shard_trace.py --report gpurun_out/${T}_shard8_ov$ov/run_kernel_trace.csv > gpurun_out/${T}_shard8_ov${ov}_timeline.txt 2>&1
  head -40 gpurun_out/${T}_shard8_ov${ov}_timeline.txt
done
