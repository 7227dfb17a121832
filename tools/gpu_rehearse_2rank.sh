# 2-rank rehearsal on a 1-GPU box: both ranks on cuda:0, gather over gloo (not a scaling
# number; checks the sharded path end to end).  bash tools/gpu_rehearse_2rank.sh <tag>
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-rXX}
export PQ_BENCH_BACKEND=gloo PQ_BENCH_SHARE_DEVICE=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_bench_2rank_gloo.log 2>&1 || { echo c3_failed; tail -20 gpurun_out/${T}_bench_2rank_gloo.log; exit 3; }
grep '^{"metric"' gpurun_out/${T}_bench_2rank_gloo.log | cut -c1-200
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --workload config5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_bench_config5_2rank_gloo.log 2>&1 || { echo c5_failed; tail -20 gpurun_out/${T}_bench_config5_2rank_gloo.log; exit 4; }
grep '^{"metric"' gpurun_out/${T}_bench_config5_2rank_gloo.log | cut -c1-200
echo rc=0
