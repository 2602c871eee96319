#!/bin/bash
# Build kernel variants HERE (CPU container):  tools/variants.sh build "<name>|<extra hipcc flags>" ...
#   -> object-triggered-3d-slam_amd/variants/libotslam_<name>.so
# Time them on the GPU box:                    tools/variants.sh bench <name> ...
#   (each: the TSDF parity tests against that library, then the bench line; OTSLAM_LIB selects the library)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mode=$1; shift
if [ "$mode" = build ]; then
  mkdir -p object-triggered-3d-slam_amd/variants
  for v in "$@"; do
    name=${v%%|*}; flags=${v#*|}
    make -j8 -C object-triggered-3d-slam_amd/csrc OUT=../variants/libotslam_$name.so BUILD=build_$name EXTRA="$flags" > /tmp/build_$name.log 2>&1 || { echo "$name build failed"; tail /tmp/build_$name.log; }
  done
  exit 0
fi
for name in "$@"; do
    timeout -k 10 300 python -u tools/with_variant.py $name -m pytest tests/test_gpu_tsdf.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/vtest_$name.log 2>&1 || { echo "$name TESTS FAILED"; tail -20 gpurun_out/vtest_$name.log; exit 1; }
  timeout -k 10 200 python3 tools/with_variant.py $name bench.py --steps 20 --warmup 2 --cpu-frames 0 --filter-frames 0 --objects 0 --hybrid-objects 0 --sustain 0 > gpurun_out/vbench_$name.log 2>&1 || { echo "$name bench failed"; tail -3 gpurun_out/vbench_$name.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/vbench_$name.log').read().strip().splitlines()[-1]);r=d['roofline'];c=d.get('color32') or {};print('$name', d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms_avg'], r['launches_per_step'], 'c32', c.get('frames_per_s'), (c.get('roofline') or {}).get('kernel_ms_avg'))"
done
