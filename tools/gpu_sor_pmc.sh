#!/bin/bash
# Counter passes over the configs[2] chain for the SOR stages (k_sor_knn / _rest / _wave): what bounds each.
# Diagnostic only (profiles/pmc_traffic.json is written by tools/pmc.sh).  TAG names the outputs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${TAG:?set TAG}
ARGS="--frames 64 --batches 64 --reps 1"
P=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
   "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum"
   "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAIT_INST_LDS")
dirs=()
for i in 0 1 2; do
  timeout -s KILL 180 rocprofv3 --pmc ${P[$i]} --kernel-trace --output-format csv -d gpurun_out/${T}_pmc$i -o run -- \
      python3 tools/filter_batch_time.py $ARGS > gpurun_out/${T}_pmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${T}_pmc$i.log; exit 1; }
  dirs+=("gpurun_out/${T}_pmc$i")
done
python3 - "${dirs[@]}" <<'PY' | tee gpurun_out/${T}_sor_pmc.txt
import importlib.util, sys
spec = importlib.util.spec_from_file_location("pp", "tools/parse_pmc.py"); pp = importlib.util.module_from_spec(spec)
spec.loader.exec_module(pp)
per = pp.load(sys.argv[1:])
for k in ("k_sor_knn", "k_sor_knn_rest", "k_sor_knn_wave"):
    c = {n: sum(v) / len(v) for n, v in per.get(k, {}).items()}
    if not c:
        continue
    print(k, {n: round(v) for n, v in sorted(c.items())})
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8.0  # per-XCD dispatch cycles (parse_pmc.py)
    w = max(c.get("SQ_WAVES", 1), 1)
    wc = c.get("SQ_WAVE_CYCLES", 0)
    if cyc and wc:
        print("   VALU issue", round(c["SQ_ACTIVE_INST_VALU"] * 4.0 / 1024.0 / cyc, 3),
              "| per wave: VALU", round(c["SQ_INSTS_VALU"] / w), "SALU", round(c.get("SQ_INSTS_SALU", 0) / w),
              "VMEM_RD", round(c["SQ_INSTS_VMEM_RD"] / w), "SMEM", round(c.get("SQ_INSTS_SMEM", 0) / w),
              "branch", round(c.get("SQ_INSTS_BRANCH", 0) / w), "LDS", round(c.get("SQ_INSTS_LDS", 0) / w),
              "| wave-cycle shares: wait_any", round(c["SQ_WAIT_ANY"] / wc, 3), "wait_inst_any",
              round(c["SQ_WAIT_INST_ANY"] / wc, 3), "active_any", round(c["SQ_ACTIVE_INST_ANY"] / wc, 3),
              "| TA", round(c.get("TA_TA_BUSY_sum", 0) / 256.0 / cyc, 3), "TD", round(c.get("TD_TD_BUSY_sum", 0) / 256.0 / cyc, 3),
              "TCC hit", round(c.get("TCC_HIT_sum", 0) / max(c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0), 1), 3),
              "| waves", round(w), "avg resident waves/CU", round(wc / cyc / 256.0, 2) if cyc else None)
PY
echo DONE
