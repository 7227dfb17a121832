# phase profile of the polish solve kernels (PQ_PROFILE build) and the round-by-round buckets
set -o pipefail
export PYTHONUNBUFFERED=1
T=r06d
PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/prof_polish.py --gcap > gpurun_out/${T}_prof_c3.log 2>&1 || { echo prof_failed; tail -20 gpurun_out/${T}_prof_c3.log; exit 3; }
PQ_PG_RT=0 PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/prof_polish.py --gcap > gpurun_out/${T}_prof_c3_rt0.log 2>&1 || { echo prof0_failed; exit 4; }
timeout -k 10 200 python -u tools/diag_rounds.py > gpurun_out/${T}_diag_rounds.log 2>&1 || { echo diag_failed; tail -20 gpurun_out/${T}_diag_rounds.log; exit 5; }
grep -A12 "grouped polish solve" gpurun_out/${T}_prof_c3.log
grep -A12 "grouped polish solve" gpurun_out/${T}_prof_c3_rt0.log
echo rc=0
