# rocprofv3 kernel stats of one short bench run -> gpurun_out/kstats.csv (+ top kernels printed)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf /tmp/kst
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d /tmp/kst -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/kstats_bench.log 2>&1 || exit 1
cp /tmp/kst/run_kernel_stats.csv gpurun_out/kstats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/kstats.csv')))
for r in rows[:28]:
    print(f"{r['Name'][:48]:48s} {int(r['Calls']):5d} {float(r['TotalDurationNs'])/3e6:8.3f} ms/step {float(r['AverageNs'])/1e3:9.1f} us")
PY
