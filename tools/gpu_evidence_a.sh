set -o pipefail
# First half of tools/gpu_evidence.sh (the GPU suite, smoke(), the config 1 / 2 / 4 / 5 bench lines,
# the drop-in phase split and the monthly run), for boxes whose call limit cannot hold both
# halves; the second half is tools/profile_round.sh.  Usage on the box: bash tools/gpu_evidence_a.sh r04Z
export PYTHONUNBUFFERED=1
T=${1:-rXX}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_full.txt 2>&1 || { echo pytest_failed; tail -30 gpurun_out/${T}_pytest_full.txt; exit 3; }
tail -2 gpurun_out/${T}_pytest_full.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke_failed; exit 4; }
for w in config1 config2 config4 config5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 > gpurun_out/${T}_bench_$w.log 2>&1 || { echo "bench $w failed"; exit 5; }
done
timeout -k 10 300 python -u tools/dropin_phases.py 3 > gpurun_out/${T}_dropin_phases.log 2>&1 || exit 6
timeout -k 10 300 python -u tools/prof_dropin.py monthly > gpurun_out/${T}_prof_dropin_monthly.log 2>&1 || exit 7
echo rc=0
