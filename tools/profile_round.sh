#!/bin/bash
# Profile collection for one round (run on the GPU box via gpurun).  Writes under gpurun_out/prof_$1.
#  1. kernel trace + stats of a short bench run
#  2. separate PMC passes (never combined with tracing): FETCH_SIZE, WRITE_SIZE, then the
#     MFMA-busy pass (SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE)
#  3. the full bench line (with CPU baseline) unless NOFULL=1
# Usage: bash tools/profile_round.sh <tag> [workload: config3 (default) | config2 | config4 | config5]
# (a non-default workload's tag should carry it, e.g. r05b_config5, so its summary is its own)
set -o pipefail
R=${1:-r01}
W=${2:-config3}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
B="bench.py --workload $W --no-cpu-baseline --no-dropin"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 $B --steps 2 --warmup 1 > $OUT/trace_bench.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/pmc_fetch -o run -- python3 $B --steps 1 --warmup 0 > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/pmc_write -o run -- python3 $B --steps 1 --warmup 0 > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -T --output-format csv -d $OUT/pmc_mfma -o run -- python3 $B --steps 1 --warmup 0 > $OUT/pmc_mfma.log 2>&1 || { echo "pmc mfma failed"; exit 1; }
if [ -z "$NOFULL" ]; then
  timeout -k 10 900 python3 bench.py --workload $W --steps 3 --warmup 1 > $OUT/bench_full.log 2>&1 || { echo "bench failed"; exit 1; }
  tail -1 $OUT/bench_full.log
fi
find $OUT -name "*.csv" | head -20
