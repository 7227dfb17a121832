# list-driven grid-stride big-LDS kernels: parity (incl. config 1/2/4), config3 + config2 + config1 bench, trace
set -o pipefail
export PYTHONUNBUFFERED=1
T=r06j
timeout -k 10 900 python -u -m pytest tests/test_polish_grouped_gpu.py tests/test_headline_parity_gpu.py tests/test_gcap_gpu.py tests/test_api_gpu.py tests/test_configs12_gpu.py tests/test_full_configs_gpu.py tests/test_polish_wide_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1 || { echo pytest_failed; tail -40 gpurun_out/${T}_pytest.txt; exit 3; }
tail -2 gpurun_out/${T}_pytest.txt
for a in "--workload config3" "--workload config3" "--workload config2" "--workload config1"; do
  n=$(echo $a | tr -d ' -')
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-dropin $a > gpurun_out/${T}_bench_$n.log 2>&1 || { echo bench_failed $a; tail -20 gpurun_out/${T}_bench_$n.log; exit 4; }
  python - <<PY
import json
d=json.loads(open("gpurun_out/${T}_bench_$n.log").read().strip().splitlines()[-1])
print("$a", round(d["value"]), round(d["ms_per_step"],3), {k: round(x*1e3,3) for k,x in d["stages_s_per_step"].items()}, d["solver"]["polish_rounds_mean"], d["solver"]["certificate"]["max_rel_stationarity"], d["solver"]["status_counts"])
PY
done
bash tools/gpu_prof.sh $T || { echo trace_failed; exit 6; }
echo rc=0
