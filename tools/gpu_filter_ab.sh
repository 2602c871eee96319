#!/bin/bash
# A/B of the configs[2] leg (bench's filtered stream only) for kernel variants; "base" = the product library
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for name in "$@"; do
  timeout -k 10 300 python3 tools/with_variant.py $name bench.py --steps 2 --warmup 1 --cpu-frames 0 --objects 0 \
      --hybrid-objects 0 --sustain 0 --color32 0 > gpurun_out/vfilt_$name.log 2>&1 || { echo "$name bench failed"; tail -3 gpurun_out/vfilt_$name.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/vfilt_$name.log').read().strip().splitlines()[-1]);f=d['filtered'];print('$name', f['ms_per_frame'], f['mpoints_per_s'])"
done
