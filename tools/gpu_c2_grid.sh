# config 2: the loose ADMM stop for tracking windows (eps_grouped_tracking) grid
set -o pipefail
T=$1
for e in 0 0.003 0.01 0 0.003 0.01; do
  timeout -k 10 300 python -u bench.py --workload config2 --steps 4 --no-cpu-baseline --no-dropin --set eps_grouped_tracking=$e > gpurun_out/${T}_b.log 2>&1 || { tail -20 gpurun_out/${T}_b.log; exit 5; }
  python3 tools/bench_summary.py "config2 eps_grouped_tracking=$e" gpurun_out/${T}_b.log | tee -a gpurun_out/${T}_grid.log
done
