# kernel trace of a short config-3 bench run (replayed steps): bash tools/gpu_trace_c3.sh <tag>
set -o pipefail
T=$1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${T} -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > gpurun_out/${T}_trace_bench.log 2>&1 || { tail -20 gpurun_out/${T}_trace_bench.log; exit 4; }
python3 tools/kseq.py gpurun_out/prof_${T}/run_kernel_trace.csv 3 | head -12
