#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_ipm_l1.py tests/test_l1.py tests/test_api_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_l1b.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_l1b.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_l1b.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/bench_l1.py --steps 2 --both 0.5,1.2 > gpurun_out/bench_l1_both.log 2>&1 || exit 2
tail -1 gpurun_out/bench_l1_both.log | cut -c1-400
