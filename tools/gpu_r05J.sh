# round-5 dev run: grouped-polish + config-2 tests, k_pg_big phase split, config-2 A/B
set -o pipefail
T=$1
timeout -k 10 600 python -u -m pytest tests/test_polish_grouped_gpu.py tests/test_configs12_gpu.py tests/test_full_configs_gpu.py::test_config2_daily_all_dates_through_backtest_run -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 3; }
tail -1 gpurun_out/${T}_pytest.txt
PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/diag_union.py > gpurun_out/${T}_diag_union.log 2>&1 || { tail -20 gpurun_out/${T}_diag_union.log; exit 6; }
grep -v amdgpu.ids gpurun_out/${T}_diag_union.log | head -8
for v in new old new old; do
  L=porqua_amd/libporqua_hip.so; [ $v = old ] && L=porqua_amd/libporqua_hip_old.so
  PQ_LIB_PATH=$L timeout -k 10 200 python -u bench.py --workload config2 --steps 5 --no-cpu-baseline --no-dropin > gpurun_out/${T}_b.log 2>&1 || { tail -20 gpurun_out/${T}_b.log; exit 5; }
  python3 tools/bench_summary.py "$v" gpurun_out/${T}_b.log | tee -a gpurun_out/${T}_ab.log
done
