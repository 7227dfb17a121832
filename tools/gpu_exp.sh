#!/bin/bash
# Short bench experiments on the GPU box (no tests): each argument is one quoted set of
# bench.py flags, e.g.  bash tools/gpu_exp.sh "--path lowrank" "--path lowrank --set refine_iters=2"
set -o pipefail
mkdir -p gpurun_out
i=0
for a in "$@"; do
    i=$((i + 1))
    timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 $a > gpurun_out/exp_$i.log 2>&1 || { echo "exp $i ($a) failed"; tail -20 gpurun_out/exp_$i.log; exit 3; }
    echo "== $a"
    tail -1 gpurun_out/exp_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"],1), {k: round(v*1e3,1) for k,v in d["stages_s_per_step"].items()}, {k: d["solver"][k] for k in ("mean_iters","polish_nfree_mean","polish_nfree_max","polish_rounds_mean","polish_rounds_max","status_counts")})'
done
