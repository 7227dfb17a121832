set -o pipefail
export PYTHONUNBUFFERED=1
for e in 2e-2 3e-2 5e-2 1e-1; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-dropin --set eps_grouped=$e > gpurun_out/r03y_bench_eg$e.log 2>&1 || exit 9
done
echo rc=$?
