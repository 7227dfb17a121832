# final check of the committed code: the whole GPU suite and smoke()
set -o pipefail
T=$1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_full.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_full.txt; exit 3; }
tail -1 gpurun_out/${T}_pytest_full.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -5 gpurun_out/${T}_smoke.log; exit 4; }
tail -1 gpurun_out/${T}_smoke.log
