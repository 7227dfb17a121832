set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-dropin > gpurun_out/r03q_bench.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_configs.py --only 12 > gpurun_out/r03q_config12_A.log 2>&1 &&
PQ_LIB_PATH=porqua_amd/libporqua_hip_b.so timeout -k 10 300 python -u tools/bench_configs.py --only 12 > gpurun_out/r03q_config12_B.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_configs.py --only 4 > gpurun_out/r03q_config4_A.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_configs12_gpu.py tests/test_window_polish_gpu.py tests/test_gpu_kernels.py tests/test_large_dense_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r03q_pytest.txt 2>&1
echo rc=$?
