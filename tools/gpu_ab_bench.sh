#!/bin/bash
# A/B timing of kernel variants (built here by tools/variants.sh build) on the headline legs only: one short bench per
# variant, "base" = the product library.  Timing only -- the product's parity is the -m gpu suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for name in "$@"; do
  timeout -k 10 200 python3 tools/with_variant.py $name bench.py --steps 20 --warmup 2 --cpu-frames 0 --filter-frames 0 \
      --objects 0 --hybrid-objects 0 --sustain 0 > gpurun_out/vbench_$name.log 2>&1 || { echo "$name bench failed"; tail -3 gpurun_out/vbench_$name.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/vbench_$name.log').read().strip().splitlines()[-1]);r=d['roofline'];c=d.get('color32') or {};print('$name', d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms_avg'], r['launches_per_step'], 'c32', c.get('frames_per_s'), (c.get('roofline') or {}).get('kernel_ms_avg'))"
done
