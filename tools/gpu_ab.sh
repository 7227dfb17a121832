#!/bin/bash
# A/B of an environment switch on the bench (no tests): bash tools/gpu_ab.sh VAR [bench args...]
set -o pipefail
mkdir -p gpurun_out
V=$1; shift
for val in 0 1; do
    env $V=$val timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" > gpurun_out/ab_$val.log 2>&1 || { echo "ab $val failed"; tail -20 gpurun_out/ab_$val.log; exit 3; }
    echo "== $V=$val"
    tail -1 gpurun_out/ab_$val.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],2), {k: round(v*1e3,2) for k,v in d["stages_s_per_step"].items()}, d["solver"]["mean_iters"], d["solver"]["status_counts"])'
done
