#!/bin/bash
# PMC diagnostics of k_sor_knn for the current library and the OT_SOR_BUF variants (filter leg only).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export KPREFIX=k_sor BENCH_ARGS="--frames 8 --steps 1 --warmup 0 --cpu-frames 0 --objects 0 --hybrid-objects 0 --filter-frames 8"
for v in base sorbuf0 sorbuf4; do
  lib=$PWD/object-triggered-3d-slam_amd/variants/libotslam_$v.so
  [ "$v" = base ] && lib=$PWD/object-triggered-3d-slam_amd/libotslam_hip.so
  echo "== $v"
  OTSLAM_LIB=$lib bash tools/pmc_diag.sh || exit 1
done
