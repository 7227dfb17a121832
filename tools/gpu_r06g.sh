# register solve ordering / restart: parity tests, bench A/B by PQ_PG_RT_MODE, phase profile
set -o pipefail
export PYTHONUNBUFFERED=1
T=r06g
timeout -k 10 600 python -u -m pytest tests/test_polish_grouped_gpu.py tests/test_headline_parity_gpu.py tests/test_gcap_gpu.py tests/test_api_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1 || { echo pytest_failed; tail -40 gpurun_out/${T}_pytest.txt; exit 3; }
tail -2 gpurun_out/${T}_pytest.txt
for v in 0 3 1 2 3 0; do
  PQ_PG_RT_MODE=$v timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-dropin > gpurun_out/${T}_bench_m$v.log 2>&1 || { echo bench_failed $v; tail -20 gpurun_out/${T}_bench_m$v.log; exit 4; }
  python - <<PY
import json
d=json.loads(open("gpurun_out/${T}_bench_m$v.log").read().strip().splitlines()[-1])
print("mode=$v", round(d["value"]), {k: round(x*1e3,3) for k,x in d["stages_s_per_step"].items()}, d["solver"]["polish_rounds_mean"], d["solver"]["certificate"]["max_rel_stationarity"], d["solver"]["status_counts"])
PY
done
PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/prof_polish.py --gcap > gpurun_out/${T}_prof_c3.log 2>&1 || { echo prof_failed; tail -20 gpurun_out/${T}_prof_c3.log; exit 5; }
grep -A14 "grouped polish solve" gpurun_out/${T}_prof_c3.log
echo rc=0
