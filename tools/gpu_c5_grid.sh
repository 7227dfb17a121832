# config 5 ADMM-stop grid (eps_grouped x min_iter_grouped): one bench line each, stage split and
# iterations / polish rounds.  Usage on the box: bash tools/gpu_c5_grid.sh <tag>
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-rXX}
CFGS=("0.5 7" "1.0 7" "0.25 7" "0.5 5" "2.0 7")
[ -n "$GRID" ] && IFS=, read -ra CFGS <<< "$GRID"   # e.g. GRID="0.6 7,0.7 7"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --workload config5 --steps 4 --no-cpu-baseline --set eps_grouped=$1 --set min_iter_grouped=$2 > gpurun_out/${T}_c5_eps$1_min$2.log 2>&1 || { echo "bench $cfg failed"; exit 5; }
  python - gpurun_out/${T}_c5_eps$1_min$2.log "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["solver"]
print(sys.argv[2], round(d["value"]), {k: round(v * 1e3, 2) for k, v in d["stages_s_per_step"].items()}, "iters", round(s["mean_iters"], 2), s["max_iters"], "rounds", round(s["polish_rounds_mean"], 2), s["polish_rounds_max"], s["status_counts"], "stat", "%.1e" % s["certificate"]["max_rel_stationarity"])
PY
done
echo rc=0
