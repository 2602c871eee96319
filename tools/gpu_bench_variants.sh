#!/bin/bash
# A/B of library variants on the headline + objects legs (no filter / hybrid / spatial legs): one short bench each
cd "$GRAFT_REPO_ROOT"
for name in "$@"; do
  timeout -k 10 300 python3 tools/with_variant.py $name bench.py --steps 50 --warmup 5 --cpu-frames 0 --filter-frames 0 \
      --hybrid-objects 0 --sustain 0 --spatial 0 > gpurun_out/vb_$name.log 2>&1 || { echo "$name bench failed"; tail -5 gpurun_out/vb_$name.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/vb_$name.log').read().strip().splitlines()[-1]);o=d.get('objects') or {};c=d.get('color32') or {};print('$name value', d['value'], 'kernel_ms', d['roofline'].get('kernel_ms_avg'), 'c32', c.get('frames_per_s'), 'objects_ms', o.get('ms'), 'single', o.get('single_object_ms'))"
done
