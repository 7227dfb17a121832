#!/bin/bash
# Round-2 GPU pass: eigen-capacitance tests, config-5 factor forms, full GPU suite, profile.
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_eigcap_gpu.py -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_eigcap.log 2>&1 || { echo "eigcap tests failed"; tail -30 gpurun_out/pytest_eigcap.log; exit 1; }
tail -3 gpurun_out/pytest_eigcap.log
timeout -k 10 300 python -u tools/bench_configs.py --only 5 --steps 1 --factor eig,chol > gpurun_out/cfg5_factor.log 2>&1 \
    || { echo "config5 failed"; tail -20 gpurun_out/cfg5_factor.log; exit 2; }
cat gpurun_out/cfg5_factor.log | grep config5
[ "$1" = "quick" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_gpu_all.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_all.log
[ $rc -le 1 ] || exit $rc
bash tools/profile_round.sh ${2:-r02g}
