set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_filters.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for occ in 5 8 10 14 20; do
  OT_SOR_OCC=$occ timeout -k 10 120 python bench.py --frames 8 --steps 1 --cpu-frames 0 > gpurun_out/sweep_$occ.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/sweep_$occ.log').read().splitlines()[-1]);print($occ, d['filtered']['ms_per_frame'], d['filtered']['mpoints_per_s'])"
done
