cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_h -o bench -- python3 bench.py \
    --objects 0 --hybrid-objects 0 --filter-frames 0 --cpu-frames 0 > gpurun_out/bench_prof_h.log 2>&1 || { tail -30 gpurun_out/bench_prof_h.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_h gpurun_out/prof_h/kernel_stats.csv
tail -1 gpurun_out/bench_prof_h.log
