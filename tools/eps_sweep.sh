set -o pipefail
mkdir -p gpurun_out
for e in 1e-3 3e-3 1e-2; do
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --set eps_abs=$e --set eps_rel=$e > gpurun_out/bench_eps_$e.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/bench_eps_$e.log').read().strip().splitlines()[-1]); s=d['solver']; print('$e', round(d['value']), round(d['ms_per_step'],2), {k: round(v*1e3,2) for k,v in d['stages_s_per_step'].items()}, s['mean_iters'], s['polish_rounds_mean'], s['status_counts'], s['certificate']['max_rel_stationarity'])"
done
PQ_LIB_PATH=$PWD/porqua_amd/libporqua_hip_prof.so timeout -k 10 200 python -u tools/prof_polish.py --gcap > gpurun_out/prof_gcap.log 2>&1; head -8 gpurun_out/prof_gcap.log
