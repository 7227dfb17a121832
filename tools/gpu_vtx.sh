#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_nfree.py > gpurun_out/diag_nfree.log 2>&1 || exit 1
grep '^{' gpurun_out/diag_nfree.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d.get('tag'), d.get('polish'), d.get('rounds_mean'), d.get('status'))"
timeout -k 10 300 python -u tools/bench_configs.py --only 5 --steps 2 > gpurun_out/cfg5.log 2>&1 || exit 2
grep '^{' gpurun_out/cfg5.log | cut -c1-500
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_all.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu_all.log | head -20; exit 3; }
