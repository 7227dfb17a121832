#!/bin/bash
# l1 GPU tests + the two l1 split bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_l1.py tests/test_ipm_l1.py tests/test_api_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_l1.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_l1.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/bench_l1.py --steps 2 --budget 0.5 > gpurun_out/l1_budget.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/bench_l1.py --steps 2 > gpurun_out/l1_cost.log 2>&1 || exit 3
for f in gpurun_out/l1_budget.log gpurun_out/l1_cost.log; do grep '^{' $f | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['workload'][:40], round(d['qps']), d['mean_iters'], d['max_iters'], round(d['polish_rounds_mean'],2), d['stage_ms'])"; done
# phase split of the grouped ADMM / polish (profiling build)
PQ_LIB_PATH=porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/prof_polish.py --gcap > gpurun_out/gcap_phases.log 2>&1 || exit 4
head -8 gpurun_out/gcap_phases.log
