#!/bin/bash
# Config-4 polish: proximal refinement steps per round vs active-set rounds (2000 dates).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/bench_configs.py --only 4 --steps 2 --dates 2000 --set refine_iters=$r > gpurun_out/refine_$r.log 2>&1 || exit 1
  grep '^{' gpurun_out/refine_$r.log | cut -c1-900
done
