# k_gcap_prep duration with its phases skipped (timing only): bash tools/gpu_prep_split.sh <tag>
set -o pipefail
T=$1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for k in 0 1 2 4 7; do
  PQ_PREP_SKIP=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${T}_$k -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-dropin > gpurun_out/${T}_$k.log 2>&1 || { tail -5 gpurun_out/${T}_$k.log; }
  echo "skip=$k $(grep k_gcap_prep gpurun_out/prof_${T}_$k/run_kernel_stats.csv | cut -d, -f1-6)"
done
