set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=r05i
timeout -k 10 1000 bash tools/pmc.sh > gpurun_out/${T}_pmc.log 2>&1 || { echo PMC_FAILED; tail -30 gpurun_out/${T}_pmc.log; exit 1; }
tail -3 gpurun_out/${T}_pmc.log
