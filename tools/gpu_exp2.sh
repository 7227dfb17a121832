#!/bin/bash
# Experiments: batched eigensolvers; slide-group size of the headline bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python -u tools/exp_eigh.py > gpurun_out/exp_eigh.log 2>&1 || { echo "eigh exp failed"; tail -20 gpurun_out/exp_eigh.log; }
tail -2 gpurun_out/exp_eigh.log
for gm in 4 12 16; do
  PQ_GROUP_MIN=$gm timeout -k 10 240 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > gpurun_out/bench_gm$gm.log 2>&1 || { echo "bench gm$gm failed"; tail -20 gpurun_out/bench_gm$gm.log; exit 1; }
  python - <<PY
import json
l=[x for x in open('gpurun_out/bench_gm$gm.log') if x.startswith('{')][-1]
d=json.loads(l)
print("gm$gm", round(d['value']), {k: round(v*1e3,3) for k,v in d['stages_s_per_step'].items()}, d['solver']['polish_rounds_mean'])
PY
done
