#!/bin/bash
# rocprofv3 PMC passes for the roofline (MI355X_MICROARCH.md HBM/rocprofv3: FETCH_SIZE and WRITE_SIZE in separate
# passes, --pmc never combined with tracing domains other than --kernel-trace).  Workloads: the headline bench leg
# (k_batch_integrate + k_export calibration) and the configs[2] batched chain (k_sor_knn).  Output:
# gpurun_out/pmc_<w>_<i>/ and profiles/pmc_traffic.json (tagged with the source hash of this build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
HEAD_ARGS="--steps 2 --warmup 1 --sustain 0 --cpu-frames 0 --filter-frames 0 --objects 0 --hybrid-objects 0 --calib"
FILT_ARGS="--frames 64 --batches 32 --reps 1"
PASSES=("FETCH_SIZE" "WRITE_SIZE"
        "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
        "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum")
dirs=()
for i in "${!PASSES[@]}"; do
  timeout -s KILL 240 rocprofv3 --pmc ${PASSES[$i]} --kernel-trace --output-format csv -d gpurun_out/pmc_h_$i -o run -- \
      python3 bench.py $HEAD_ARGS > gpurun_out/pmc_h_$i.log 2>&1 || { echo "pass h$i failed"; tail -5 gpurun_out/pmc_h_$i.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc ${PASSES[$i]} --kernel-trace --output-format csv -d gpurun_out/pmc_f_$i -o run -- \
      python3 tools/filter_batch_time.py $FILT_ARGS > gpurun_out/pmc_f_$i.log 2>&1 || { echo "pass f$i failed"; tail -5 gpurun_out/pmc_f_$i.log; exit 1; }
  dirs+=("gpurun_out/pmc_h_$i" "gpurun_out/pmc_f_$i")
done
python3 tools/parse_pmc.py "${dirs[@]}" > gpurun_out/pmc_traffic.json && cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json && python3 -c "
import json; d=json.load(open('profiles/pmc_traffic.json')); print(json.dumps({k: d[k] for k in ('source_hash','config','kernels_traffic')}, indent=1))"
