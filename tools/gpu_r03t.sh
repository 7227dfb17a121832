set -o pipefail
export PYTHONUNBUFFERED=1
for e in 2e-2 5e-2 1e-1; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-dropin --set eps_abs=$e --set eps_rel=$e > gpurun_out/r03t_bench_eps$e.log 2>&1 || exit 9
done
for e in 2e-3 1e-2 2e-2; do
  timeout -k 10 200 python -u tools/bench_configs.py --only 12 --set eps_abs=$e --set eps_rel=$e > gpurun_out/r03t_config12_eps$e.log 2>&1 || exit 8
  timeout -k 10 200 python -u tools/bench_configs.py --only 4 --set eps_abs=$e --set eps_rel=$e > gpurun_out/r03t_config4_eps$e.log 2>&1 || exit 7
done
echo rc=$?
