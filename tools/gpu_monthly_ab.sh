# monthly-run (13 dates, config 2 shape) timings under factor variants, after the given tests
set -o pipefail
T=$1; shift
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 3; }
  tail -1 gpurun_out/${T}_pytest.txt
fi
for v in "default" "PQ_GCAP_FACTOR=large" "PQ_FACTOR_SK=0" "default"; do
  E=""; [ "$v" != default ] && E="$v"
  env $E timeout -k 10 200 python -u tools/prof_dropin.py monthly > gpurun_out/${T}_m.log 2>&1 || { tail -20 gpurun_out/${T}_m.log; exit 5; }
  echo "$v $(grep 'run s' gpurun_out/${T}_m.log)" | tee -a gpurun_out/${T}_monthly_ab.log
done
