#!/bin/bash
# the filtered leg's ms/frame with the legs in either order (objects first / filtered first).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r02o}
for order in "filtered,objects" "objects,filtered"; do
  OT_BENCH_ORDER=$order timeout -k 10 300 python3 bench.py --steps 20 --cpu-frames 0 --sustain 0 --color64 0 --hybrid-objects 0 > gpurun_out/${TAG}_order_${order/,/_}.log 2>&1 || { echo "order $order failed"; tail -5 gpurun_out/${TAG}_order_${order/,/_}.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_order_${order/,/_}.log').read().strip().splitlines()[-1]);print('$order', 'filtered', d['filtered']['ms_per_frame'], 'objects', d['objects']['ms'], 'headline', d['value'])"
done
