# Round-5 evidence, second half: short config-3 / config-2 A/Bs of the working tree against
# porqua_amd/libporqua_hip_old.so, then tools/profile_round.sh for config 3 (trace, PMC passes,
# the full bench line with the CPU baseline) and the config-2 trace / PMC passes.
# Usage on the box: bash tools/gpu_evidence_r05b.sh r05Z
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-rXX}
if [ -f porqua_amd/libporqua_hip_old.so ]; then
  for w in config3 config2; do
    for v in new old new old; do
      L=porqua_amd/libporqua_hip.so; [ $v = old ] && L=porqua_amd/libporqua_hip_old.so
      PQ_LIB_PATH=$L timeout -k 10 200 python -u bench.py --workload $w --steps 6 --no-cpu-baseline --no-dropin > gpurun_out/${T}_ab_b.log 2>&1 || { tail -20 gpurun_out/${T}_ab_b.log; exit 5; }
      python3 tools/bench_summary.py "$w $v" gpurun_out/${T}_ab_b.log | tee -a gpurun_out/${T}_ab.log
    done
  done
fi
bash tools/profile_round.sh ${T} > gpurun_out/${T}_profile_round.log 2>&1 || { tail -20 gpurun_out/${T}_profile_round.log; exit 6; }
tail -3 gpurun_out/${T}_profile_round.log
NOFULL=1 bash tools/profile_round.sh ${T}_config2 config2 > gpurun_out/${T}_config2_profile.log 2>&1 || { tail -20 gpurun_out/${T}_config2_profile.log; exit 7; }
echo rc=0
