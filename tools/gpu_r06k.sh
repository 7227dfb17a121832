# big-free-set launches first; host planning fast paths: tests, bench config3/config2, drop-in phases, trace
set -o pipefail
export PYTHONUNBUFFERED=1
T=r06k
timeout -k 10 900 python -u -m pytest tests/test_polish_grouped_gpu.py tests/test_headline_parity_gpu.py tests/test_api_gpu.py tests/test_configs12_gpu.py tests/test_graph_mode_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1 || { echo pytest_failed; tail -40 gpurun_out/${T}_pytest.txt; exit 3; }
tail -2 gpurun_out/${T}_pytest.txt
for a in "--workload config3" "--workload config3" "--workload config2"; do
  n=$(echo $a | tr -d ' -')
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-dropin $a > gpurun_out/${T}_bench_$n.log 2>&1 || { echo bench_failed $a; tail -20 gpurun_out/${T}_bench_$n.log; exit 4; }
  python - <<PY
import json
d=json.loads(open("gpurun_out/${T}_bench_$n.log").read().strip().splitlines()[-1])
print("$a", round(d["value"]), round(d["ms_per_step"],3), {k: round(x*1e3,3) for k,x in d["stages_s_per_step"].items()}, d["solver"]["polish_rounds_mean"], d["stage_rates"]["gram_tflops"])
PY
done
timeout -k 10 200 python -u tools/dropin_phases.py 5 > gpurun_out/${T}_dropin_phases.log 2>&1 || { echo ph_failed; tail -30 gpurun_out/${T}_dropin_phases.log; exit 6; }
grep -E "plain run|top-level|stage|solve shard|finish|drop-in solve stages" gpurun_out/${T}_dropin_phases.log
bash tools/gpu_prof.sh $T || { echo trace_failed; exit 7; }
echo rc=0
