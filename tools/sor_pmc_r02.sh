#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export KPREFIX=k_sor BENCH_ARGS="--frames 8 --steps 1 --warmup 0 --cpu-frames 0 --objects 0 --hybrid-objects 0 --filter-frames 8 --filter-streams 1"
timeout -k 10 200 bash tools/pmc_diag.sh > gpurun_out/sor_pmc.json 2> gpurun_out/sor_pmc.err || { tail -20 gpurun_out/sor_pmc.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sor_kt -o b -- python3 bench.py $BENCH_ARGS > gpurun_out/sor_kt.log 2>&1 || exit 1
echo DONE
