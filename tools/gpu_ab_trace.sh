# tests + A/B vs libporqua_hip_old.so + a kernel trace of the new library: bash tools/gpu_ab_trace.sh <tag> [tests...]
set -o pipefail
T=$1; shift
bash tools/gpu_ab_lib.sh $T "$@" || exit $?
bash tools/gpu_trace_c3.sh $T
