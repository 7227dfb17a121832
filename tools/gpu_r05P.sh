# 32-date groups for the wide ADMM form: gcap / config-4 GPU tests, then config 4 A/B by
# PQ_GCAP32_WIDE (1 new, 0 old) on the same library
set -o pipefail
T=$1
timeout -k 10 900 python -u -m pytest tests/test_gcap_gpu.py tests/test_full_configs_gpu.py::test_config4_full_batch_certified_and_matches_oracle tests/test_polish_wide_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 3; }
tail -1 gpurun_out/${T}_pytest.txt
for v in new old new old; do
  E=1; [ $v = old ] && E=0
  PQ_GCAP32_WIDE=$E timeout -k 10 300 python -u bench.py --workload config4 --steps 3 --no-cpu-baseline --no-dropin > gpurun_out/${T}_b.log 2>&1 || { tail -20 gpurun_out/${T}_b.log; exit 5; }
  python3 tools/bench_summary.py "config4 $v" gpurun_out/${T}_b.log | tee -a gpurun_out/${T}_ab.log
done
