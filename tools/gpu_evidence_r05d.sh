# Round-5 final check after the 32-date wide form: the GPU suite, smoke(), the default bench
# line (config 3) and config 4's line with their CPU baselines, config 4's trace / PMC passes.
# Usage on the box: bash tools/gpu_evidence_r05d.sh r05Zd
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-rXX}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_full.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_full.txt; exit 3; }
tail -1 gpurun_out/${T}_pytest_full.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -5 gpurun_out/${T}_smoke.log; exit 4; }
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || { tail -20 gpurun_out/${T}_bench.log; exit 5; }
python3 tools/bench_summary.py config3 gpurun_out/${T}_bench.log
timeout -k 10 400 python -u bench.py --workload config4 --steps 3 > gpurun_out/${T}_bench_config4.log 2>&1 || { tail -20 gpurun_out/${T}_bench_config4.log; exit 6; }
python3 tools/bench_summary.py config4 gpurun_out/${T}_bench_config4.log
NOFULL=1 bash tools/profile_round.sh ${T}_config4 config4 > gpurun_out/${T}_config4_profile.log 2>&1 || { tail -20 gpurun_out/${T}_config4_profile.log; exit 7; }
echo rc=0
