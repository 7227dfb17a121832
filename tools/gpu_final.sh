#!/bin/bash
# Round-2 closing pass: headline profile (trace + PMC) and bench line, secondary bench lines.
set -o pipefail
mkdir -p gpurun_out
bash tools/profile_round.sh ${1:-r02h} || exit 1
timeout -k 10 400 python -u tools/bench_configs.py --steps 2 > gpurun_out/bench_configs.log 2>&1 || { echo "configs failed"; tail -5 gpurun_out/bench_configs.log; exit 2; }
grep '^{' gpurun_out/bench_configs.log | cut -c1-400
timeout -k 10 300 python -u tools/bench_lad.py > gpurun_out/bench_lad.log 2>&1 || { echo "lad failed"; tail -5 gpurun_out/bench_lad.log; exit 3; }
tail -1 gpurun_out/bench_lad.log | cut -c1-300
timeout -k 10 300 python -u tools/bench_l1.py --steps 2 --both 0.5,1.2 > gpurun_out/bench_l1_both.log 2>&1 || { echo "l1 both failed"; exit 4; }
tail -1 gpurun_out/bench_l1_both.log | cut -c1-300
