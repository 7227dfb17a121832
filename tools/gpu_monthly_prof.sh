# kernel trace of the reference notebook's monthly run (13 dates, config 2 shape): bash tools/gpu_monthly_prof.sh <tag>
set -o pipefail
T=$1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python3 -u tools/prof_dropin.py monthly > gpurun_out/${T}_monthly.log 2>&1 || { tail -20 gpurun_out/${T}_monthly.log; exit 3; }
grep "run s" gpurun_out/${T}_monthly.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_${T}_monthly -o run -- python3 tools/prof_dropin.py monthly > gpurun_out/${T}_monthly_trace.log 2>&1 || { tail -20 gpurun_out/${T}_monthly_trace.log; exit 4; }
echo done
