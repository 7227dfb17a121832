# k_admm_gcap / polish phase clocks at config 3 (profiling build): bash tools/gpu_gcap_phases.sh
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-rXX}
PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so timeout -k 10 300 python -u tools/prof_polish.py --gcap > gpurun_out/${T}_prof_gcap.log 2>&1 || { echo prof_failed; tail -20 gpurun_out/${T}_prof_gcap.log; exit 3; }
head -30 gpurun_out/${T}_prof_gcap.log
echo rc=0
