#!/bin/bash
# GPU suite + drop-in profile + short bench (each step time-limited, stop at first failure)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_gpu_all.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_all.log
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu_all.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/prof_dropin.py mv3 > gpurun_out/prof_dropin_mv3.log 2>&1 || exit 2
head -3 gpurun_out/prof_dropin_mv3.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || exit 3
python -c "
import json; l=[x for x in open('gpurun_out/bench_quick.log') if x.startswith('{')][-1]; d=json.loads(l)
print(round(d['value']), d['end_to_end']['qps'], {k: round(v*1e3,3) for k,v in d['stages_s_per_step'].items()})"
