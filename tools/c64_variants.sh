cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in ${VS:-base w5 w6 w7 w8}; do
  timeout -k 10 200 python3 tools/with_variant.py $v bench.py --steps 20 --cpu-frames 0 --sustain 0 --filter-frames 0 --hybrid-objects 0 --objects 0 > gpurun_out/c64_$v.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/c64_$v.log').read().strip().splitlines()[-1]);print('$v', d['value'], d['color64']['frames_per_s'], d['color64']['kernel_ms_avg'])"
done
