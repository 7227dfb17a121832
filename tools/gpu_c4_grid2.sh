# config 4: eps_grouped_tracking_wide grid around the default 1e-2
set -o pipefail
T=$1
for e in 0.01 0.015 0.02 0.01 0.015 0.02; do
  timeout -k 10 300 python -u bench.py --workload config4 --steps 3 --no-cpu-baseline --no-dropin --set eps_grouped_tracking_wide=$e > gpurun_out/${T}_b.log 2>&1 || { tail -20 gpurun_out/${T}_b.log; exit 5; }
  python3 tools/bench_summary.py "config4 eps_grouped_tracking_wide=$e" gpurun_out/${T}_b.log | tee -a gpurun_out/${T}_grid.log
done
