#!/bin/bash
# GPU suite, then configs 4 / 5 and the headline after the per-date polish's two-step refinement.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_all.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu_all.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/bench_configs.py --only 5 --steps 2 > gpurun_out/cfg5.log 2>&1 || exit 2
grep '^{' gpurun_out/cfg5.log | cut -c1-700
timeout -k 10 300 python -u tools/bench_configs.py --only 4 --steps 2 > gpurun_out/cfg4.log 2>&1 || exit 3
grep '^{' gpurun_out/cfg4.log | cut -c1-700
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || exit 4
python3 -c "
import json; l=[x for x in open('gpurun_out/bench_quick.log') if x.startswith('{')][-1]; d=json.loads(l)
print(round(d['value']), d['end_to_end']['qps'], {k: round(v*1e3,3) for k,v in d['stages_s_per_step'].items()})"
