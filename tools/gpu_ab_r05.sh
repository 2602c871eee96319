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
