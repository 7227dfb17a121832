set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-dropin > gpurun_out/r03u_bench.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_configs.py --only 12 > gpurun_out/r03u_config12.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_configs.py --only 4 > gpurun_out/r03u_config4.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_headline_parity_gpu.py tests/test_polish_grouped_gpu.py tests/test_gcap_gpu.py tests/test_polish_wide_gpu.py tests/test_configs12_gpu.py tests/test_full_configs_gpu.py tests/test_api_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03u_pytest.txt 2>&1
echo rc=$?
