# Kernel trace + stats of a short default bench run (no PMC), for the per-kernel split and the
# step timeline: bash tools/gpu_prof.sh <tag> [bench args...]
#   -> gpurun_out/<tag>_kernel_stats.csv, <tag>_kernel_trace.csv, <tag>_trace_bench.log
#   (locally: python tools/kseq.py gpurun_out/<tag>_kernel_trace.csv 1 > ..._step_timeline.log)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf /tmp/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d /tmp/prof_$TAG -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin "$@" > gpurun_out/${TAG}_trace_bench.log 2>&1 || exit 1
cp /tmp/prof_$TAG/run_kernel_stats.csv gpurun_out/${TAG}_kernel_stats.csv
cp /tmp/prof_$TAG/run_kernel_trace.csv gpurun_out/${TAG}_kernel_trace.csv
echo prof_ok
