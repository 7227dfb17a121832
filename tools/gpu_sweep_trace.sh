# sweep dev run plus the kernel stats of the isolated ADMM run: bash tools/gpu_sweep_trace.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash tools/gpu_sweep_dev.sh r06L || exit 3
rm -rf /tmp/prof_r06L
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d /tmp/prof_r06L -o run -- python3 tools/exp_sweep_admm.py 12 --sweep-only > gpurun_out/r06L_trace.log 2>&1 || exit 4
cp /tmp/prof_r06L/run_kernel_stats.csv gpurun_out/r06L_kernel_stats.csv
grep -E "k_sw_pass|k_sw_mid" gpurun_out/r06L_kernel_stats.csv | cut -d, -f1-4
echo rc=0
