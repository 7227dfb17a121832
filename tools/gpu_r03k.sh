set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03K_pytest_full.txt 2>&1 || { echo pytest_failed; exit 3; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03K_smoke.log 2>&1 || { echo smoke_failed; exit 4; }
timeout -k 10 300 python -u tools/bench_configs.py --only 12 > gpurun_out/r03K_config12.log 2>&1 || exit 5
timeout -k 10 300 python -u tools/bench_configs.py --only 4 > gpurun_out/r03K_config4.log 2>&1 || exit 6
bash tools/profile_round.sh r03K > gpurun_out/r03K_profile_round.log 2>&1
echo rc=$?
