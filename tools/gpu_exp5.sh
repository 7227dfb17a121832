#!/bin/bash
# config-5 initial-rho grid (rho0_rel x rho0_qrel)
set -o pipefail
mkdir -p gpurun_out/exp5
for a in 4; do for b in 30 60 100 300; do
  timeout -k 10 200 python -u tools/bench_configs.py --only 5 --steps 1 --set rho0_rel=$a --set rho0_qrel=$b > gpurun_out/exp5/c5_${a}_${b}.log 2>&1 || { echo "fail $a $b"; exit 1; }
  python3 -c "
import json; l=[x for x in open('gpurun_out/exp5/c5_${a}_${b}.log') if x.startswith('{')][-1]; d=json.loads(l)
print('rho0_rel $a rho0_qrel $b', round(d['qps']), d['mean_iters'], d['max_iters'], d['stage_ms'], d['status_counts'])"
done; done
