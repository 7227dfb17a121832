# The whole GPU suite and one headline bench line: bash tools/gpu_suite.sh <tag>
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${1}_pytest_full.txt 2>&1 || { echo pytest_failed; exit 3; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${1}_smoke.log 2>&1 || { echo smoke_failed; exit 4; }
timeout -k 10 200 python -u bench.py > gpurun_out/${1}_bench.log 2>&1
echo rc=$?
