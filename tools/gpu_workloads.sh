# Sweep / tracking tests and the config2 / config5 bench lines (1 rank and a 2-rank gloo
# rehearsal on one GPU): bash tools/gpu_workloads.sh <tag>
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_cov_at_size_gpu.py tests/test_jacobi_gpu.py tests/test_active_set_polish.py tests/test_large_dense_gpu.py tests/test_full_configs_gpu.py tests/test_eigcap_gpu.py tests/test_large_n_gpu.py tests/test_configs12_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${1}_pytest_workloads.txt 2>&1 || { echo pytest_failed; exit 3; }
timeout -k 10 300 python -u bench.py --workload config5 --steps 3 > gpurun_out/${1}_bench_config5.log 2>&1 || { echo c5_failed; exit 4; }
timeout -k 10 300 python -u bench.py --workload config2 --steps 3 > gpurun_out/${1}_bench_config2.log 2>&1 || { echo c2_failed; exit 5; }
PQ_BENCH_BACKEND=gloo PQ_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python -u bench.py --workload config5 --gpus 2 --steps 2 > gpurun_out/${1}_bench_config5_2rank_gloo.log 2>&1 || { echo c5x2_failed; exit 6; }
echo rc=$?
