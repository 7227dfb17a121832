# the loose stop for wide tracking problems: wide / config-4 / gcap GPU tests, then config 4's
# bench line with its CPU baseline and config 2's line (unaffected: one general row)
set -o pipefail
export PYTHONUNBUFFERED=1
T=$1
timeout -k 10 900 python -u -m pytest tests/test_polish_wide_gpu.py tests/test_gcap_gpu.py tests/test_full_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 3; }
tail -1 gpurun_out/${T}_pytest.txt
timeout -k 10 400 python -u bench.py --workload config4 --steps 3 > gpurun_out/${T}_bench_config4.log 2>&1 || { tail -20 gpurun_out/${T}_bench_config4.log; exit 5; }
python3 tools/bench_summary.py config4 gpurun_out/${T}_bench_config4.log
timeout -k 10 300 python -u bench.py --workload config2 --steps 3 --no-cpu-baseline --no-dropin > gpurun_out/${T}_bench_config2.log 2>&1 || { tail -20 gpurun_out/${T}_bench_config2.log; exit 6; }
python3 tools/bench_summary.py config2 gpurun_out/${T}_bench_config2.log
