#!/bin/bash
# GPU suite (optional), then a kernel trace of a short bench run (tools/kseq.py reads it)
set -o pipefail
mkdir -p gpurun_out/tr
if [ "$1" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
      > gpurun_out/pytest_gpu_all.log 2>&1; rc=$?
  tail -2 gpurun_out/pytest_gpu_all.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu_all.log | head -20; exit 1; }
fi
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/tr/*
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin > gpurun_out/tr/bench.log 2>&1 || exit 2
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || exit 3
python3 -c "
import json; l=[x for x in open('gpurun_out/bench_quick.log') if x.startswith('{')][-1]; d=json.loads(l)
print(round(d['value']), d['end_to_end']['qps'], {k: round(v*1e3,3) for k,v in d['stages_s_per_step'].items()})"
