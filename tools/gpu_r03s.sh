set -o pipefail
export PYTHONUNBUFFERED=1
for e in 2e-3 3e-3 5e-3 1e-2; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-dropin --set eps_abs=$e --set eps_rel=$e > gpurun_out/r03s_bench_eps$e.log 2>&1 || exit 9
done
PQ_PG_SOLVE_NW=4 timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-dropin > gpurun_out/r03s_bench_nw4.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-dropin --set alpha=1.8 > gpurun_out/r03s_bench_alpha18.log 2>&1
echo rc=$?
