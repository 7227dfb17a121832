# round-5 diagnostics: the monthly run's kernel trace and the polish phase / inner-step counters
# at config 3 (profile build): bash tools/gpu_diag_r05.sh <tag>
set -o pipefail
T=$1
PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/prof_polish.py --gcap > gpurun_out/${T}_prof_c3.log 2>&1 || { tail -20 gpurun_out/${T}_prof_c3.log; exit 6; }
grep -v amdgpu.ids gpurun_out/${T}_prof_c3.log | tail -16
bash tools/gpu_monthly_prof.sh $T || exit 7
