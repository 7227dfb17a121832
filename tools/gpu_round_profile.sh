# Round profile: profile_round.sh for config 3 (trace, PMC passes, full bench line), then the
# k_admm_gcap / polish phase clocks of the profiling build.  bash tools/gpu_round_profile.sh <tag>
set -o pipefail
T=${1:-rXX}
bash tools/profile_round.sh $T || exit 3
bash tools/gpu_gcap_phases.sh $T || exit 4
echo rc=0
