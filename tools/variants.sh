#!/bin/bash
# Build-and-bench kernel variants on the GPU box: each entry is "<name>|<extra hipcc flags>".
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in "$@"; do
  name=${v%%|*}; flags=${v#*|}
  make -C object-triggered-3d-slam_amd/csrc clean > /dev/null && make -j16 -C object-triggered-3d-slam_amd/csrc EXTRA="$flags" > gpurun_out/build_$name.log 2>&1 || { echo "$name build failed"; continue; }
  timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-frames 0 > gpurun_out/bench_$name.log 2>&1 || { echo "$name bench failed"; tail -3 gpurun_out/bench_$name.log; break; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/bench_$name.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$name', d['value'], d['ms_per_step'], r['kernel_ms_avg'], r['launches_per_step'])"
done
