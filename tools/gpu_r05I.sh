# config 2 after the big group form: k_pg_big phase split (profile build) and a kernel trace
set -o pipefail
T=$1
PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/diag_union.py > gpurun_out/${T}_diag_union.log 2>&1 || { tail -20 gpurun_out/${T}_diag_union.log; exit 6; }
grep -v amdgpu.ids gpurun_out/${T}_diag_union.log | tail -12
bash tools/gpu_prof.sh ${T}_config2 --workload config2 || exit 7
echo prof_done
