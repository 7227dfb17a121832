# Development run on the GPU box: bash tools/gpu_dev.sh <tag> "<test files>" "<bench arg sets separated by ;>"
# Each step under its own time limit; stops at the first failure.
set -o pipefail
export PYTHONUNBUFFERED=1
TAG=$1
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest $2 -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.txt 2>&1 || { echo pytest_failed; tail -30 gpurun_out/${TAG}_pytest.txt; exit 3; }
  tail -3 gpurun_out/${TAG}_pytest.txt
fi
i=0
IFS=';' read -ra SETS <<< "$3"
for a in "${SETS[@]}"; do
  [ -z "$a" ] && continue
  timeout -k 10 300 python -u bench.py $a > gpurun_out/${TAG}_bench_$i.log 2>&1 || { echo "bench $i failed: $a"; tail -30 gpurun_out/${TAG}_bench_$i.log; exit 4; }
  tail -c 600 gpurun_out/${TAG}_bench_$i.log
  i=$((i+1))
done
echo rc=0
