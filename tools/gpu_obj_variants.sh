#!/bin/bash
# configs[3] one-object phases and the configs[1] headline for the product library and the variants in $VARIANTS
# (tools/variants.sh build): TSDF parity tests first for each variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-objv}
for v in base ${VARIANTS:-}; do
  if [ "$v" != base ]; then
    timeout -k 10 300 python -u tools/with_variant.py $v -m pytest tests/test_gpu_tsdf.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_t_$v.log 2>&1 || { echo "$v TESTS FAILED"; tail -20 gpurun_out/${TAG}_t_$v.log; exit 1; }
  fi
  timeout -k 10 200 python3 -u tools/with_variant.py $v tools/single_object_phases.py > gpurun_out/${TAG}_ph_$v.log 2>&1 || { tail -5 gpurun_out/${TAG}_ph_$v.log; exit 1; }
  timeout -k 10 200 python3 tools/with_variant.py $v bench.py --steps 50 --warmup 3 --cpu-frames 0 --filter-frames 0 --hybrid-objects 0 --sustain 0 --color32 0 > gpurun_out/${TAG}_b_$v.log 2>&1 || { tail -3 gpurun_out/${TAG}_b_$v.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/${TAG}_b_$v.log').read().strip().splitlines()[-1]);r=d['roofline'];o=d['objects']
ph=open('gpurun_out/${TAG}_ph_$v.log').read().split('\n')
print('$v', 'value', d['value'], 'kernel', r['kernel_ms_avg'], 'objects', o['ms'], 'single', o['single_object_ms'], '|', [l.strip() for l in ph if l.startswith('integrate') or l.startswith('total')])"
done
