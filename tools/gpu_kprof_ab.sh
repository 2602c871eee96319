#!/bin/bash
# Per-kernel durations (rocprofv3 kernel trace) of the configs[2] filter batch for the product library ("base") and
# each variant in $VARIANTS: gpurun_out/${TAG}_kp_<v>.csv, the top kernels printed.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-kp}
for v in base ${VARIANTS:-}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_kp_$v -o fb -- python3 tools/with_variant.py $v tools/filter_batch_time.py --frames 64 --batches 32 --reps 2 > gpurun_out/${TAG}_kp_$v.log 2>&1 || { tail -20 gpurun_out/${TAG}_kp_$v.log; exit 1; }
  python3 tools/prof_summary.py gpurun_out/${TAG}_kp_$v gpurun_out/${TAG}_kp_$v.csv > /dev/null
  echo "== $v"; python3 - gpurun_out/${TAG}_kp_$v.csv <<'PY'
import csv, sys
r = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: -float(x["TotalDurationNs"]))
tot = sum(float(x["TotalDurationNs"]) for x in r)
print("total ms", round(tot / 1e6, 3))
for x in r[:12]:
    print(f'{x["Name"][:60]:60s} {x["Calls"]:>5s} {float(x["AverageNs"])/1e3:9.1f} us')
PY
  rm -rf gpurun_out/${TAG}_kp_$v
done
