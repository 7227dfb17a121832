#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_lad_gpu.py tests/test_ipm_l1.py tests/test_api_gpu.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_lad.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_lad.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_lad.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/bench_lad.py --dates 4749 > gpurun_out/bench_lad.log 2>&1 || exit 2
tail -1 gpurun_out/bench_lad.log | cut -c1-300
