set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_polish_grouped_gpu.py tests/test_headline_parity_gpu.py tests/test_window_polish_gpu.py tests/test_nan_backtest_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03L_pytest.txt 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-dropin > gpurun_out/r03L_bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r03L -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin > gpurun_out/r03L_trace_bench.log 2>&1
echo rc=$?
