# config 3: the loose stop's iteration floor (min_iter_grouped) grid, two passes
set -o pipefail
T=$1
for m in 8 6 7 9 8 6 7 9; do
  timeout -k 10 300 python -u bench.py --steps 6 --no-cpu-baseline --no-dropin --set min_iter_grouped=$m > gpurun_out/${T}_b.log 2>&1 || { tail -20 gpurun_out/${T}_b.log; exit 5; }
  python3 tools/bench_summary.py "config3 min_iter_grouped=$m" gpurun_out/${T}_b.log | tee -a gpurun_out/${T}_grid.log
done
