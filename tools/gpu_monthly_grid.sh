# monthly-run settings grid (tools/monthly_grid.py): bash tools/gpu_monthly_grid.sh <tag> '<json>' ...
set -o pipefail
T=$1; shift
timeout -k 10 300 python -u tools/monthly_grid.py "$@" > gpurun_out/${T}_monthly_grid.log 2>&1 || { tail -20 gpurun_out/${T}_monthly_grid.log; exit 3; }
grep -v amdgpu.ids gpurun_out/${T}_monthly_grid.log
