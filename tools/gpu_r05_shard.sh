#!/bin/bash
# Sharded-integrate check: TSDF / shard / bench-scale parity tests, 1/4 and 1/8 shards' step times for the integrate
# granularities and front-end modes, one 1/8 shard's timeline, and the bench's measured per-rank steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
T=${TAG:?set TAG}
timeout -k 10 600 python -u -m pytest tests/test_gpu_tsdf.py tests/test_gpu_shard.py tests/test_gpu_bench_scale.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for w in 4 8; do for fine in 0 1; do for ov in 1 0; do
  timeout -k 10 120 python3 -u tools/shard_trace.py --world $w --overlap $ov --fine $fine > gpurun_out/${T}_s${w}_f${fine}_o${ov}.log 2>&1 \
      || { echo SHARD_FAILED; tail -20 gpurun_out/${T}_s${w}_f${fine}_o${ov}.log; exit 1; }
  grep "ms/step" gpurun_out/${T}_s${w}_f${fine}_o${ov}.log
done; done; done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_shard8 -o run -- python3 -u \
    tools/shard_trace.py --world 8 > gpurun_out/${T}_shard8.log 2>&1 || { echo SHARDTRACE_FAILED; tail -20 gpurun_out/${T}_shard8.log; exit 1; }
python3 tools/shard_trace.py --report gpurun_out/${T}_shard8/run_kernel_trace.csv > gpurun_out/${T}_shard8_timeline.txt 2>&1
head -24 gpurun_out/${T}_shard8_timeline.txt
A="--filter-frames 0 --objects 0 --hybrid-objects 0 --cpu-frames 0 --sustain 0 --color32 0 --steps 100"
timeout -k 10 300 python3 bench.py $A > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/${T}_bench.log; exit 1; }
TAG=$T python3 - <<'PY'
import json, os
d = json.loads(open(f"gpurun_out/{os.environ['TAG']}_bench.log").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_avg"])
print(json.dumps(d["spatial_amdahl"]["measured"]["worlds"]))
PY
