#!/bin/bash
# Diagnostic PMC passes for k_batch_integrate (KPREFIX selects other kernels; VARIANT a variant library; SCRIPT
# another driver script than bench.py, with BENCH_ARGS its arguments) (one rocprofv3 run per pass; --pmc never combined with tracing
# domains other than --kernel-trace).  Output: gpurun_out/diag_<i>/ and a per-kernel summary on stdout.
set -e
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGS=${BENCH_ARGS:-"--steps 1 --warmup 0 --cpu-frames 0 --filter-frames 0"}
PASSES=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVES"
  "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
  "SQ_INST_CYCLES_VMEM_RD SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES TCP_TCC_READ_REQ_LATENCY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAVES"
)
dirs=()
for i in "${!PASSES[@]}"; do
  timeout -s KILL 150 rocprofv3 --pmc ${PASSES[$i]} --kernel-trace --output-format csv -d gpurun_out/diag_$i -o run -- \
      python3 tools/with_variant.py ${VARIANT:-base} ${SCRIPT:-bench.py} $ARGS > gpurun_out/diag_$i.log 2>&1
  dirs+=("gpurun_out/diag_$i")
done
python3 - "${dirs[@]}" <<'PY'
import csv, glob, os, sys, json
from collections import defaultdict
per = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "").split("(")[0].split("::")[-1]
            per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
pref = os.environ.get("KPREFIX", "k_batch")
out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items() if k.startswith(pref)}
print(json.dumps(out, indent=1))
PY
