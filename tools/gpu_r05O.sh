# round-5 dev run: polish / config-2 tests, then config-2 A/B of the working tree against HEAD
set -o pipefail
T=$1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1 || { tail -40 gpurun_out/${T}_pytest.txt; exit 3; }
tail -1 gpurun_out/${T}_pytest.txt
for v in new old new old; do
  L=porqua_amd/libporqua_hip.so; [ $v = old ] && L=porqua_amd/libporqua_hip_old.so
  PQ_LIB_PATH=$L timeout -k 10 200 python -u bench.py --workload config2 --steps 6 --no-cpu-baseline --no-dropin > gpurun_out/${T}_b.log 2>&1 || { tail -20 gpurun_out/${T}_b.log; exit 5; }
  python3 tools/bench_summary.py "config2 $v" gpurun_out/${T}_b.log | tee -a gpurun_out/${T}_ab.log
done
timeout -k 10 300 python -u tools/monthly_grid.py '{"small_batch": 0}' '{"eps_grouped_tracking_small": 0.3}' > gpurun_out/${T}_monthly_grid.log 2>&1 || { tail -20 gpurun_out/${T}_monthly_grid.log; exit 6; }
grep -v amdgpu.ids gpurun_out/${T}_monthly_grid.log
