#!/bin/bash
# rocprofv3 PMC passes for the rooflines (MI355X_MICROARCH.md HBM/rocprofv3: FETCH_SIZE and WRITE_SIZE in separate
# passes, --pmc never combined with tracing domains other than --kernel-trace).  Workloads:
#   c  : tools/fetch_calib (known-byte reads / writes per access pattern: the FETCH / WRITE corrections)
#   h64: the headline bench leg at colour precision 64 (k_batch_integrate<true>)
#   h32: the same at colour precision 32 (k_batch_integrate<false>), FETCH / WRITE only
#   f  : the configs[2] batched chain (k_sor_knn), 64-frame batches as bench.py times them
# Output: gpurun_out/pmc_<w>_<i>/ and profiles/pmc_traffic.json (tagged with the source hash of this build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
HEAD_ARGS="--steps 2 --warmup 1 --sustain 0 --cpu-frames 0 --filter-frames 0 --objects 0 --hybrid-objects 0 --color32 0 --shard-steps 0"
FILT_ARGS="--frames 128 --batches 64 --reps 1"  # the bench times 64-frame batches (--filter-batch 64)
TRAFFIC=("FETCH_SIZE" "WRITE_SIZE")
DIAG=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
      "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum")
run() {  # run <dir> <counters> -- <cmd...>
  local d=$1 c=$2; shift 3
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/$d -o run -- "$@" \
      > gpurun_out/$d.log 2>&1 || { echo "pass $d failed"; tail -5 gpurun_out/$d.log; exit 1; }
}
[ -x tools/fetch_calib ] || /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o tools/fetch_calib tools/fetch_calib.hip || exit 1
cal=(); dirs=()
for i in 0 1; do
  run pmc_c_$i "${TRAFFIC[$i]}" -- ./tools/fetch_calib 1024; cal+=("gpurun_out/pmc_c_$i")
  run pmc_h64_$i "${TRAFFIC[$i]}" -- python3 bench.py $HEAD_ARGS --color-bits 64; dirs+=("gpurun_out/pmc_h64_$i")
  run pmc_h32_$i "${TRAFFIC[$i]}" -- python3 bench.py $HEAD_ARGS --color-bits 32; dirs+=("gpurun_out/pmc_h32_$i")
  run pmc_f_$i "${TRAFFIC[$i]}" -- python3 tools/filter_batch_time.py $FILT_ARGS; dirs+=("gpurun_out/pmc_f_$i")
done
for i in 0 1; do
  run pmc_h64_d$i "${DIAG[$i]}" -- python3 bench.py $HEAD_ARGS --color-bits 64; dirs+=("gpurun_out/pmc_h64_d$i")
  run pmc_f_d$i "${DIAG[$i]}" -- python3 tools/filter_batch_time.py $FILT_ARGS; dirs+=("gpurun_out/pmc_f_d$i")
done
python3 tools/parse_pmc.py --calib "${cal[@]}" -- "${dirs[@]}" > gpurun_out/pmc_traffic.json && \
  cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json && python3 -c "
import json; d=json.load(open('profiles/pmc_traffic.json')); print(json.dumps({k: d[k] for k in ('source_hash','calibration','kernels_traffic')}, indent=1))"
