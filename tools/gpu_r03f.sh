#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r03f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 200 python tools/chain_mesh_diag.py || exit 1
timeout -k 10 200 python3 tools/single_object_phases.py || exit 1
bash tools/gpu_ab_bench.sh base || exit 1
echo DONE
