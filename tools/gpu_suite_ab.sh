# the whole GPU suite, then an A/B of the built library against libporqua_hip_old.so (config 3)
set -o pipefail
T=$1
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_full.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest_full.txt; exit 3; }
tail -1 gpurun_out/${T}_pytest_full.txt
bash tools/gpu_ab_lib.sh $T
