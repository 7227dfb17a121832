# config-2 kernel trace (replayed steps) + config-3 ADMM phase profile (PQ_PROFILE build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r05r_c2 -o run -- python3 bench.py --workload config2 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin > gpurun_out/r05r_c2_trace.log 2>&1 || exit 4
PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/prof_polish.py --gcap > gpurun_out/r05r_prof_c3.log 2>&1 || exit 5
grep -v amdgpu.ids gpurun_out/r05r_prof_c3.log | head -12
