# register solve on its own side stream: bench config3 x2 + trace
set -o pipefail
export PYTHONUNBUFFERED=1
T=r06l
for a in "--workload config3" "--workload config3"; do
  n=$(echo $a | tr -d ' -')
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-dropin $a > gpurun_out/${T}_bench_$n.log 2>&1 || { echo bench_failed $a; tail -20 gpurun_out/${T}_bench_$n.log; exit 4; }
  python - <<PY
import json
d=json.loads(open("gpurun_out/${T}_bench_$n.log").read().strip().splitlines()[-1])
print("$a", round(d["value"]), round(d["ms_per_step"],3), {k: round(x*1e3,3) for k,x in d["stages_s_per_step"].items()}, d["solver"]["polish_rounds_mean"])
PY
done
bash tools/gpu_prof.sh $T || { echo trace_failed; exit 7; }
python tools/kseq.py gpurun_out/${T}_kernel_trace.csv 1 > gpurun_out/${T}_timeline.log 2>&1 || true
grep -E "k_pg_solve|k_pg_big|k_pg_init|step span" gpurun_out/${T}_timeline.log | head -30
echo rc=0
