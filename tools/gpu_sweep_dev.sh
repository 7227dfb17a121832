# sweep ADMM development run: parity tests, isolated timing, phase clocks (profiling build)
# bash tools/gpu_sweep_dev.sh <tag>
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-rXX}
timeout -k 10 300 python -u -m pytest tests/test_sweep_admm_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1; rc=$?; tail -2 gpurun_out/${T}_pytest.txt; [ $rc -le 1 ] || exit 3
timeout -k 10 240 python -u tools/exp_sweep_admm.py 12 --sweep-only > gpurun_out/${T}_exp.log 2>&1 || { echo exp_failed; exit 4; }
grep "^sweep" gpurun_out/${T}_exp.log
if [ -f porqua_amd/libporqua_hip_swprof.so ] && [ -z "$NOPROF" ]; then
  PQ_LIB_PATH=porqua_amd/libporqua_hip_swprof.so timeout -k 10 240 python -u tools/exp_sweep_admm.py 12 --sweep-only --prof > gpurun_out/${T}_prof.log 2>&1 || { echo prof_failed; exit 5; }
  grep -E "phase" gpurun_out/${T}_prof.log
fi
echo rc=0
