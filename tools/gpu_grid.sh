# A/B grid of engine settings on the headline bench: bash tools/gpu_grid.sh <tag> "<set args 1>" "<set args 2>" ...
set -o pipefail
export PYTHONUNBUFFERED=1
tag=$1; shift; i=0
for a in "$@"; do
  timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-dropin $a > gpurun_out/${tag}_grid$i.log 2>&1 || exit 9
  echo "$a" >> gpurun_out/${tag}_grid$i.log; i=$((i+1))
done
echo rc=$?
