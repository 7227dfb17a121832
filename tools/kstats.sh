# rocprofv3 kernel stats of one short bench run: bash tools/kstats.sh <tag> [bench args...]
# -> gpurun_out/<tag>_kstats.csv, top kernels printed per step (steps = k_admm_gcap calls)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf /tmp/kst_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d /tmp/kst_$TAG -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin "$@" > gpurun_out/${TAG}_kstats_bench.log 2>&1 || exit 1
cp /tmp/kst_$TAG/run_kernel_stats.csv gpurun_out/${TAG}_kstats.csv
python3 - gpurun_out/${TAG}_kstats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = max(1, sum(int(r['Calls']) for r in rows if r['Name'].startswith('k_admm_gcap')))
print("steps (k_admm_gcap calls):", steps)
for r in rows[:30]:
    print(f"{r['Name'][:56]:56s} {int(r['Calls']) / steps:7.1f}/step {float(r['TotalDurationNs']) / steps / 1e6:8.3f} ms/step {float(r['AverageNs']) / 1e3:9.1f} us")
PY
