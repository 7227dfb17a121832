# register-tile polish solve: grouped-polish + headline parity tests, then bench A/B by PQ_PG_RT
set -o pipefail
export PYTHONUNBUFFERED=1
T=r06b
timeout -k 10 600 python -u -m pytest tests/test_polish_grouped_gpu.py tests/test_headline_parity_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1 || { echo pytest_failed; tail -40 gpurun_out/${T}_pytest.txt; exit 3; }
tail -3 gpurun_out/${T}_pytest.txt
for v in 0 3 4 0 3 4; do
  PQ_PG_RT=$v timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-dropin > gpurun_out/${T}_bench_rt$v.log 2>&1 || { echo bench_failed $v; tail -20 gpurun_out/${T}_bench_rt$v.log; exit 4; }
  python - <<PY
import json
d=json.loads(open("gpurun_out/${T}_bench_rt$v.log").read().strip().splitlines()[-1])
print("rt=$v", round(d["value"]), {k: round(x*1e3,3) for k,x in d["stages_s_per_step"].items()}, d["solver"]["polish_rounds_mean"], d["solver"]["certificate"]["max_rel_stationarity"], d["solver"]["status_counts"])
PY
done
echo rc=0
