#!/bin/bash
# Counters of the marching-cubes emission halves (two-stream form, so each half is its own kernel) on one object:
# one pass per counter set, --pmc with --kernel-trace only.  TAG names the outputs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:?set TAG}
SETS=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
      "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum" "FETCH_SIZE" "WRITE_SIZE")
for i in 0 1 2 3; do
  timeout -s KILL 120 rocprofv3 --pmc ${SETS[$i]} --kernel-trace --output-format csv -d gpurun_out/${T}_mcpmc_$i -o run -- \
      python3 tools/single_object_trace.py --fork > gpurun_out/${T}_mcpmc_$i.log 2>&1 || { echo PMC_FAILED $i; tail -5 gpurun_out/${T}_mcpmc_$i.log; exit 1; }
done
python3 - <<PY
import csv, glob, collections
T="${T}"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/{T}_mcpmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if "k_mc_" in k:
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k, {c: round(sum(v) / len(v), 1) for c, v in sorted(cs.items())})
PY
echo DONE
