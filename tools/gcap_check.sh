# group-capacitance ADMM check: gcap + grouped-polish + headline parity tests, one bench line, phase profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gcap_gpu.py tests/test_polish_grouped_gpu.py tests/test_headline_parity_gpu.py > gpurun_out/t_gc.log 2>&1 || { tail -30 gpurun_out/t_gc.log; exit 1; }
tail -2 gpurun_out/t_gc.log
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_gc.log 2>&1 || { tail -20 gpurun_out/bench_gc.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_gc.log').read().strip().splitlines()[-1]); s=d['solver']; print(round(d['value']), round(d['ms_per_step'],2), {k: round(v*1e3,2) for k,v in d['stages_s_per_step'].items()}, s['mean_iters'], s['polish_rounds_mean'], s['status_counts'], s['certificate']['max_rel_stationarity'])"
PQ_LIB_PATH=$PWD/porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/prof_polish.py --gcap > gpurun_out/prof_gcap.log 2>&1; head -9 gpurun_out/prof_gcap.log
