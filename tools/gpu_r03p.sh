set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_polish_grouped_gpu.py tests/test_headline_parity_gpu.py tests/test_polish_wide_gpu.py tests/test_nan_backtest_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r03p_pytest.txt 2>&1 &&
for nw in 0 1 2 4; do PQ_PG_SOLVE_NW=$nw timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-dropin > gpurun_out/r03p_bench_nw$nw.log 2>&1 || exit 9; done &&
PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/prof_polish.py --gcap > gpurun_out/r03p_prof_polish.log 2>&1
echo rc=$?
