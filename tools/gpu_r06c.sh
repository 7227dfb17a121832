# kernel trace of the default bench (register-tile polish solve), then K1 covariance lines
set -o pipefail
export PYTHONUNBUFFERED=1
T=r06c
bash tools/gpu_prof.sh $T || { echo prof_failed; tail -20 gpurun_out/${T}_trace_bench.log; exit 3; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dropin --with-cov > gpurun_out/${T}_bench_withcov.log 2>&1 || { echo cov_failed; tail -20 gpurun_out/${T}_bench_withcov.log; exit 4; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dropin --with-cov --no-slide --dates 1024 > gpurun_out/${T}_bench_withcov_noslide.log 2>&1 || { echo cov2_failed; tail -20 gpurun_out/${T}_bench_withcov_noslide.log; exit 5; }
for f in withcov withcov_noslide; do python - <<PY
import json
d=json.loads(open("gpurun_out/${T}_bench_$f.log").read().strip().splitlines()[-1])
print("$f", round(d["value"]), {k: round(x*1e3,3) for k,x in d["stages_s_per_step"].items()}, d["stage_rates"]["cov_syrk_tflops"], d["stage_rates"]["cov_write_gbs"])
PY
done
timeout -k 10 200 python -u tools/dropin_phases.py 5 > gpurun_out/${T}_dropin_phases.log 2>&1 || { echo ph_failed; tail -30 gpurun_out/${T}_dropin_phases.log; exit 6; }
echo rc=0
