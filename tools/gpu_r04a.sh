#!/bin/bash
# r04a: the new timed-state / IEEE-kernel parity tests first, then every -m gpu test, the default bench line, the
# self-launched 2-rank rehearsal (bench.py --gpus 2, no torch.distributed.run) and the VALU-rate microbenchmark.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:-r04a}
timeout -k 10 120 ./tools/valu_rate > gpurun_out/${T}_valu_rate.log 2>&1 || { echo VALU_FAILED; cat gpurun_out/${T}_valu_rate.log; exit 1; }
cat gpurun_out/${T}_valu_rate.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_scale.py tests/test_gpu_filter_batch.py tests/test_gpu_tsdf.py \
  tests/test_gpu_mesh.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_new_tests.log 2>&1 \
  || { echo NEW_TESTS_FAILED; tail -60 gpurun_out/${T}_new_tests.log; exit 1; }
tail -2 gpurun_out/${T}_new_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_bench_scale.py --deselect tests/test_gpu_filter_batch.py --deselect tests/test_gpu_tsdf.py \
  --deselect tests/test_gpu_mesh.py > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/${T}_bench.log; exit 1; }
tail -1 gpurun_out/${T}_bench.log | cut -c1-600
OT_BENCH_BACKEND=gloo OT_BENCH_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 1 --cpu-frames 0 \
  --filter-frames 0 > gpurun_out/${T}_self2.log 2>&1 || { echo SELF2_FAILED; tail -30 gpurun_out/${T}_self2.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/${T}_self2.log') if l.startswith('{')][-1])
print('self-launched', d['n_gpus'], d['value'], d['spatial']['mesh_matches_unsharded'], d['objects']['ms'])"
echo DONE
