#!/bin/bash
# Grouped polish: refinement steps per round vs rounds (headline shape, config 5).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  PQ_LIB_PATH=$PWD/porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/prof_polish.py --gcap --refine=$r > gpurun_out/prof_g_refine_$r.log 2>&1 || exit 1
  grep -E "rounds mean|stage polish|stage admm" gpurun_out/prof_g_refine_$r.log
  timeout -k 10 200 python -u tools/bench_configs.py --only 5 --steps 2 --set refine_iters=$r > gpurun_out/cfg5_refine_$r.log 2>&1 || exit 2
  grep '^{' gpurun_out/cfg5_refine_$r.log | cut -c1-700
done
