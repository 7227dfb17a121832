# polish A/B: grouped-polish tests, then config-3 bench lines alternating an environment knob
# bash tools/gpu_polish_ab.sh <tag> "<ENV=a>" "<ENV=b>"
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-rXX}; A=$2; B=$3
timeout -k 10 600 python -u -m pytest tests/test_polish_grouped_gpu.py tests/test_headline_parity_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1; rc=$?; tail -2 gpurun_out/${T}_pytest.txt; [ $rc -le 1 ] || exit 3
for i in 0 1 2; do
  for V in "$A" "$B"; do
    env $V timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-dropin > gpurun_out/${T}_bench_${i}_${V//=/_}.log 2>&1 || { echo bench_failed; exit 4; }
    python -c "import json; d=json.loads(open('gpurun_out/${T}_bench_${i}_${V//=/_}.log').read().strip().splitlines()[-1]); print('$V', round(d['value']), {k: round(x*1e3,3) for k,x in d['stages_s_per_step'].items()}, round(d['solver']['polish_rounds_mean'],2))"
  done
done
echo rc=0
