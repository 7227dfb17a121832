set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/diag_gform.py > gpurun_out/r03J_diag_gform.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_polish_grouped_gpu.py tests/test_headline_parity_gpu.py tests/test_window_polish_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03J_pytest.txt 2>&1 &&
for g in 3 1 2 5; do PQ_PG_GFORM=$g timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-dropin > gpurun_out/r03J_bench_gform$g.log 2>&1 || exit 9; done
echo rc=$?
