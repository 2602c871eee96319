#!/bin/bash
# Sharded-integrate check: TSDF / shard / bench-scale parity tests, one 1/8 shard's timeline with and without the
# double-buffered front end, and the bench's measured per-rank steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
T=${TAG:?set TAG}
timeout -k 10 600 python -u -m pytest tests/test_gpu_tsdf.py tests/test_gpu_shard.py tests/test_gpu_bench_scale.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
for ov in 1 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_shard8_ov$ov -o run -- python3 -u \
      tools/shard_trace.py --world 8 --overlap $ov > gpurun_out/${T}_shard8_ov$ov.log 2>&1 || { echo SHARDTRACE_FAILED; tail -20 gpurun_out/${T}_shard8_ov$ov.log; exit 1; }
  grep "ms/step" gpurun_out/${T}_shard8_ov$ov.log
  python3 tools/shard_trace.py --report gpurun_out/${T}_shard8_ov$ov/run_kernel_trace.csv > gpurun_out/${T}_shard8_ov${ov}_timeline.txt 2>&1
  head -24 gpurun_out/${T}_shard8_ov${ov}_timeline.txt
done
A="--filter-frames 0 --objects 0 --hybrid-objects 0 --cpu-frames 0 --sustain 0 --color32 0 --steps 100"
timeout -k 10 300 python3 bench.py $A > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/${T}_bench.log; exit 1; }
TAG=$T python3 - <<'PY'
import json, os
d = json.loads(open(f"gpurun_out/{os.environ['TAG']}_bench.log").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_avg"])
print(json.dumps(d["spatial_amdahl"]["measured"]["worlds"]))
PY
