# Round-5 last evidence: the GPU suite and smoke() on the final commit, config 4's trace / PMC
# passes at its loose stop.  Usage on the box: bash tools/gpu_evidence_r05e.sh r05Ze
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-rXX}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_full.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_full.txt; exit 3; }
tail -1 gpurun_out/${T}_pytest_full.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -5 gpurun_out/${T}_smoke.log; exit 4; }
tail -1 gpurun_out/${T}_smoke.log
NOFULL=1 bash tools/profile_round.sh ${T}_config4 config4 > gpurun_out/${T}_config4_profile.log 2>&1 || { tail -20 gpurun_out/${T}_config4_profile.log; exit 7; }
echo rc=0
