# grid cap of the <=128 LDS bucket (PQ_PG_LDS_GRID) A/B, trace
set -o pipefail
export PYTHONUNBUFFERED=1
T=r06n
for v in 64 0 64 0; do
  PQ_PG_LDS_GRID=$v timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-dropin > gpurun_out/${T}_bench_g$v.log 2>&1 || { echo bench_failed; exit 4; }
  python - <<PY
import json
d=json.loads(open("gpurun_out/${T}_bench_g$v.log").read().strip().splitlines()[-1])
print("grid=$v", round(d["value"]), round(d["ms_per_step"],3), {k: round(x*1e3,3) for k,x in d["stages_s_per_step"].items()})
PY
done
PQ_PG_LDS_GRID=64 bash tools/gpu_prof.sh ${T}g64 || { echo trace_failed; exit 7; }
python tools/kseq.py gpurun_out/${T}g64_kernel_trace.csv 1 > gpurun_out/${T}g64_timeline.log 2>&1 || true
grep -E "k_pg_solve|k_pg_big|k_pg_init|step span" gpurun_out/${T}g64_timeline.log | head -16
echo rc=0
