#!/bin/bash
# Collect rocprofv3 PMC counters for the headline bench, one counter group per pass (MI355X_MICROARCH.md:
# FETCH_SIZE and WRITE_SIZE cannot share a pass; no --sys-trace with --pmc).  Output: gpurun_out/pmc_<i>/.
set -e
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGS=${BENCH_ARGS:-"--steps 1 --warmup 0 --cpu-frames 0 --filter-frames 0 --calib"}
i=0
for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  timeout -k 10 240 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d gpurun_out/pmc_$i -o run -- \
      python3 bench.py $ARGS > gpurun_out/pmc_$i.log 2>&1
  i=$((i+1))
done
python3 tools/parse_pmc.py gpurun_out/pmc_0 gpurun_out/pmc_1 gpurun_out/pmc_2 gpurun_out/pmc_3
