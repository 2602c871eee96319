#!/bin/bash
# A round's records on one box: tools/gpu_final.sh (tests, smoke, bench, kernel stats, one object's timeline), then
# tools/pmc.sh (same-hash PMC traffic), then the bench line again with the fresh PMC file (physical roofline frac).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:?set TAG}
TAG=$T bash tools/gpu_final.sh || exit 1
timeout -k 10 1500 bash tools/pmc.sh > gpurun_out/${T}_pmc.log 2>&1 || { echo PMC_FAILED; tail -30 gpurun_out/${T}_pmc.log; exit 1; }
tail -5 gpurun_out/${T}_pmc.log
timeout -k 10 400 python3 bench.py > gpurun_out/${T}_bench2.log 2>&1 || { echo BENCH2_FAILED; tail -30 gpurun_out/${T}_bench2.log; exit 1; }
tail -1 gpurun_out/${T}_bench2.log > gpurun_out/${T}_bench2.json
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_bench2.json')); r=d['roofline']
print('value', d['value'], 'frac', r.get('frac'), 'eff', r.get('frac_effective'), 'valu', r.get('valu_busy_frac'), 'td', r.get('td_busy_frac'))
print('filtered', d['filtered']['ms_per_frame'], d['filtered']['kernel_roofline'])
print('objects', d['objects']['ms'], d['objects']['single_object_ms'], d['objects']['objects_over_single'])"
