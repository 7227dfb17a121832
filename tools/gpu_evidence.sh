set -o pipefail
# Round evidence on one GPU box: the whole GPU suite, smoke(), configs 1/2 and 4, then
# tools/profile_round.sh (kernel trace + PMC passes + the default bench line).  Usage on the box:
#   bash tools/gpu_evidence.sh r03K   ->  gpurun_out/r03K_* and gpurun_out/prof_r03K/
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${1:-rXX}_pytest_full.txt 2>&1 || { echo pytest_failed; exit 3; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${1:-rXX}_smoke.log 2>&1 || { echo smoke_failed; exit 4; }
timeout -k 10 300 python -u tools/bench_configs.py --only 12 > gpurun_out/${1:-rXX}_config12.log 2>&1 || exit 5
timeout -k 10 300 python -u tools/bench_configs.py --only 4 > gpurun_out/${1:-rXX}_config4.log 2>&1 || exit 6
bash tools/profile_round.sh ${1:-rXX} > gpurun_out/${1:-rXX}_profile_round.log 2>&1
echo rc=$?
