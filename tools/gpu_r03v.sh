set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03v_pytest_full.txt 2>&1
echo pytest_rc=$?
timeout -k 10 300 python -u tools/bench_configs.py --only 12 > gpurun_out/r03v_config12.log 2>&1 &&
bash tools/profile_round.sh r03v > gpurun_out/r03v_profile_round.log 2>&1
echo rc=$?
