#!/bin/bash
# Closing pass of the session: GPU suite, smoke, default bench line (driver form), profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_all.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu_all.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 2; }
tail -2 gpurun_out/smoke.log
bash tools/profile_round.sh ${1:-r02k} || exit 3
timeout -k 10 400 python -u tools/bench_configs.py --steps 2 > gpurun_out/bench_configs.log 2>&1 || exit 4
grep '^{' gpurun_out/bench_configs.log | cut -c1-200
