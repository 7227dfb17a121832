set -o pipefail
# Round evidence on one GPU box: the whole GPU suite, smoke(), the bench lines of configs 2, 4
# and 5, the drop-in phase split, then tools/profile_round.sh (kernel trace + PMC passes + the
# default bench line).  Usage on the box:
#   bash tools/gpu_evidence.sh r04Z  ->  gpurun_out/r04Z_* and gpurun_out/prof_r04Z/
export PYTHONUNBUFFERED=1
T=${1:-rXX}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_full.txt 2>&1 || { echo pytest_failed; tail -30 gpurun_out/${T}_pytest_full.txt; exit 3; }
tail -2 gpurun_out/${T}_pytest_full.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke_failed; exit 4; }
for w in config2 config4 config5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 > gpurun_out/${T}_bench_$w.log 2>&1 || { echo "bench $w failed"; exit 5; }
done
timeout -k 10 300 python -u tools/dropin_phases.py 3 > gpurun_out/${T}_dropin_phases.log 2>&1 || exit 6
timeout -k 10 300 python -u tools/prof_dropin.py monthly > gpurun_out/${T}_prof_dropin_monthly.log 2>&1 || exit 7
bash tools/profile_round.sh ${T} > gpurun_out/${T}_profile_round.log 2>&1
echo rc=$?
