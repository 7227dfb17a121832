set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_l1.py tests/test_ipm_l1.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05s_pytest_l1.txt 2>&1 || { tail -40 gpurun_out/r05s_pytest_l1.txt; exit 3; }
tail -1 gpurun_out/r05s_pytest_l1.txt
timeout -k 10 300 python -u tools/bench_l1.py --both 0.5,1.3 > gpurun_out/r05s_bench_l1_both_seg.log 2>&1 || { tail -20 gpurun_out/r05s_bench_l1_both_seg.log; exit 4; }
tail -c 1500 gpurun_out/r05s_bench_l1_both_seg.log
