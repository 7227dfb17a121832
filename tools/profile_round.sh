#!/bin/bash
# Profile collection for one round (run on the GPU box via gpurun).  Writes under gpurun_out/prof_$1.
#  1. kernel trace + stats of a short bench run
#  2. separate PMC passes (never combined with tracing): FETCH_SIZE, WRITE_SIZE, then the
#     MFMA-busy pass (SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE)
#  3. the full bench line (with CPU baseline)
set -o pipefail
R=${1:-r01}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin > $OUT/trace_bench.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-dropin > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-dropin > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -T --output-format csv -d $OUT/pmc_mfma -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-dropin > $OUT/pmc_mfma.log 2>&1 || { echo "pmc mfma failed"; exit 1; }
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > $OUT/bench_full.log 2>&1 || { echo "bench failed"; exit 1; }
find $OUT -name "*.csv" | head -20
tail -1 $OUT/bench_full.log
