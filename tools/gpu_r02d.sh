#!/bin/bash
# Round-2 GPU pass: API tests, drop-in bench, sweep variants, gcap phase split.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_api_gpu.py tests/test_configs12_gpu.py tests/test_nan_backtest_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/api_tests.log 2>&1 || { echo "api tests failed"; tail -20 gpurun_out/api_tests.log; exit 1; }
tail -2 gpurun_out/api_tests.log
timeout -k 10 300 python -u tools/bench_dropin.py --profile > gpurun_out/dropin.log 2> gpurun_out/dropin_prof.log || { echo "dropin failed"; exit 1; }
tail -1 gpurun_out/dropin.log
ND=16 timeout -k 10 300 python -u tools/exp_sweep.py > gpurun_out/exp_sweep.log 2>&1 || { echo "sweep failed"; tail -5 gpurun_out/exp_sweep.log; exit 1; }
cat gpurun_out/exp_sweep.log | grep shared
PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so timeout -k 10 300 python -u tools/prof_polish.py --gcap > gpurun_out/prof_gcap.log 2>&1 || { echo "prof failed"; exit 1; }
head -12 gpurun_out/prof_gcap.log
