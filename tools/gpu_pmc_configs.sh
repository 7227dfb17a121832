# Round-5 evidence: pivot-chain microbenchmark, then the PMC / trace passes of the given
# workloads (tools/profile_round.sh, NOFULL) -- bash tools/gpu_pmc_configs.sh <tag> <workload>...
set -o pipefail
T=$1; shift
if [ -x tools/chainbench ]; then
  timeout -k 10 60 tools/chainbench > gpurun_out/${T}_chainbench.log 2>&1 || { cat gpurun_out/${T}_chainbench.log; exit 2; }
  cat gpurun_out/${T}_chainbench.log
fi
for W in "$@"; do
  NOFULL=1 bash tools/profile_round.sh ${T}_$W $W > gpurun_out/${T}_$W.log 2>&1 || { tail -20 gpurun_out/${T}_$W.log; exit 3; }
  echo "$W done"
done
