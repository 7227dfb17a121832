# Round-5 final config-3 profile on the committed code: the gcap GPU tests, then
# tools/profile_round.sh (trace, PMC passes, the full bench line).  Usage: bash tools/gpu_evidence_r05c.sh r05ZZ
set -o pipefail
export PYTHONUNBUFFERED=1
T=${1:-rXX}
timeout -k 10 600 python -u -m pytest tests/test_gcap_gpu.py tests/test_headline_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.txt 2>&1 || { tail -30 gpurun_out/${T}_pytest.txt; exit 3; }
tail -1 gpurun_out/${T}_pytest.txt
bash tools/profile_round.sh ${T} > gpurun_out/${T}_profile_round.log 2>&1 || { tail -20 gpurun_out/${T}_profile_round.log; exit 6; }
tail -1 gpurun_out/prof_${T}/bench_full.log | cut -c1-200
echo rc=0
