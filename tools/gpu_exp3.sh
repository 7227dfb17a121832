#!/bin/bash
# ADMM stopping tolerance x initial rho grid on the headline bench (stages, rounds, certificate)
set -o pipefail
mkdir -p gpurun_out/exp3
for eps in 1e-3 2e-3; do
  for r0 in 1.6 1.7 1.8; do
    timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dropin \
      --set eps_abs=$eps --set eps_rel=$eps --set alpha=$r0 > gpurun_out/exp3/b_${eps}_${r0}.log 2>&1 || { echo "fail $eps $r0"; exit 1; }
    python3 - <<PY
import json
l=[x for x in open('gpurun_out/exp3/b_${eps}_${r0}.log') if x.startswith('{')][-1]; d=json.loads(l); s=d['solver']
print("eps ${eps} alpha ${r0}", round(d['value']), {k: round(v*1e3,2) for k,v in d['stages_s_per_step'].items()},
      "iters", s['mean_iters'], s['max_iters'], "rounds", round(s['polish_rounds_mean'],2), s['polish_rounds_max'],
      "cert", s['certificate']['max_violation'], s['certificate']['max_rel_stationarity'], s['status_counts'])
PY
  done
done
