# config 2 (the SPTR replication workload): k_pg_big's phase split (profile build) and the free
# set / group union sizes: bash tools/gpu_diag_big.sh <tag>
set -o pipefail
T=$1
PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/diag_union.py > gpurun_out/${T}_diag_union.log 2>&1 || { tail -20 gpurun_out/${T}_diag_union.log; exit 6; }
grep -v amdgpu.ids gpurun_out/${T}_diag_union.log | tail -24
