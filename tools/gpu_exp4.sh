#!/bin/bash
# turnover-budget split: ADMM settings grid (iterations, QPs/s)
set -o pipefail
mkdir -p gpurun_out/exp4
i=0
for args in "" "--no-gcap" "--no-gcap --set rho0_rel=4"; do
  i=$((i+1))
  timeout -k 10 200 python -u tools/bench_l1.py --steps 2 --budget 0.5 $args > gpurun_out/exp4/l1_$i.log 2>&1 || { echo "fail $args"; tail -5 gpurun_out/exp4/l1_$i.log; exit 1; }
  echo "[$args] $(grep '^{' gpurun_out/exp4/l1_$i.log | tail -1 | cut -c1-260)"
done
