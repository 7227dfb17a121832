#!/bin/bash
# One GPU-box pass: parity tests, then short bench runs of both solve paths.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh [bench args...]
# Stops at the first GPU step that crashes, times out or fails.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for p in lowrank dense; do
    timeout -k 10 300 python -u bench.py --path $p --no-cpu-baseline "$@" > gpurun_out/bench_$p.log 2>&1 || { echo "bench $p failed"; tail -20 gpurun_out/bench_$p.log; exit 3; }
    tail -1 gpurun_out/bench_$p.log
done
