# A/B of the working-tree library against porqua_amd/libporqua_hip_old.so on config 3 and
# config 2 after the given GPU tests: bash tools/gpu_ab2.sh <tag> [pytest files...]
set -o pipefail
T=$1; shift
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 3; }
  tail -1 gpurun_out/${T}_pytest.txt
fi
for w in config3 config2; do
  for v in new old new old; do
    L=porqua_amd/libporqua_hip.so; [ $v = old ] && L=porqua_amd/libporqua_hip_old.so
    PQ_LIB_PATH=$L timeout -k 10 200 python -u bench.py --workload $w --steps 6 --no-cpu-baseline --no-dropin > gpurun_out/${T}_b.log 2>&1 || { tail -20 gpurun_out/${T}_b.log; exit 5; }
    python3 tools/bench_summary.py "$w $v" gpurun_out/${T}_b.log | tee -a gpurun_out/${T}_ab.log
  done
done
