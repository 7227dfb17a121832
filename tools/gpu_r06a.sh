set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py > gpurun_out/r06a_bench.log 2>&1 || { echo bench_failed; tail -30 gpurun_out/r06a_bench.log; exit 3; }
timeout -k 10 200 python -u tools/dropin_phases.py 5 > gpurun_out/r06a_dropin_phases.log 2>&1 || { echo ph_failed; tail -30 gpurun_out/r06a_dropin_phases.log; exit 4; }
timeout -k 10 200 python -u tools/prof_dropin.py mv3 > gpurun_out/r06a_prof_dropin.log 2>&1 || { echo prof_failed; tail -30 gpurun_out/r06a_prof_dropin.log; exit 5; }
timeout -k 10 200 python -u tools/prof_dropin.py monthly > gpurun_out/r06a_prof_monthly.log 2>&1 || { echo m_failed; exit 6; }
echo rc=0
