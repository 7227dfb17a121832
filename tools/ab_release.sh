# A/B of Settings.polish_release_rel on config 3 (bash tools/ab_release.sh on the GPU box)
set -o pipefail
for v in 0 0.001 0.01 0.1 0; do
  timeout -k 10 200 python -u bench.py --steps 5 --no-cpu-baseline --no-dropin --set polish_release_rel=$v > gpurun_out/r05q_b.log 2>&1 || { tail -20 gpurun_out/r05q_b.log; exit 5; }
  python3 tools/bench_summary.py "release=$v" gpurun_out/r05q_b.log
done
