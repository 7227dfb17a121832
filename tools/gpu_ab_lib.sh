# A/B of the built library against porqua_amd/libporqua_hip_old.so on config 3 (+ given tests):
# bash tools/gpu_ab_lib.sh <tag> [pytest files...]
set -o pipefail
T=$1; shift
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 3; }
  tail -1 gpurun_out/${T}_pytest.txt
fi
for v in new old new old; do
  L=porqua_amd/libporqua_hip.so; [ $v = old ] && L=porqua_amd/libporqua_hip_old.so
  PQ_LIB_PATH=$L timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline --no-dropin ${BENCH_ARGS} > gpurun_out/${T}_b.log 2>&1 || { tail -20 gpurun_out/${T}_b.log; exit 5; }
  python3 tools/bench_summary.py "$v" gpurun_out/${T}_b.log | tee -a gpurun_out/${T}_ab.log
done
if [ -n "$PROF" ] && [ -f porqua_amd/libporqua_hip_prof.so ]; then
  PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/prof_polish.py --gcap > gpurun_out/${T}_prof_c3.log 2>&1 || exit 6
  grep -v amdgpu.ids gpurun_out/${T}_prof_c3.log | head -40
fi
