#!/bin/bash
# k_sor_knn kernel time per library variant (rocprofv3 kernel trace of the configs[2] leg).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd); cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for v in "$@"; do
    rm -rf gpurun_out/st_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/st_$v -o b -- \
    python3 tools/with_variant.py $v bench.py --frames 8 --steps 1 --warmup 0 --cpu-frames 0 --objects 0 --hybrid-objects 0 --filter-frames 32 \
    > gpurun_out/st_$v.log 2>&1 || { tail -5 gpurun_out/st_$v.log; exit 1; }
  python3 tools/prof_summary.py gpurun_out/st_$v gpurun_out/st_$v/ks.csv > /dev/null
  echo "$v $(grep -h 'k_sor_knn' gpurun_out/st_$v/ks.csv | cut -d, -f2,4 | head -1)  filtered: $(grep '^{' gpurun_out/st_$v.log | tail -1 | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["filtered"]["ms_per_frame"])')"
done
