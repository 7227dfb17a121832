# Run one gpurun command, retrying only while the pool has no free slot or box (exit code 3, or
# a "transient" verdict: nothing ran, nothing charged); any other outcome ends it.
# Usage: bash tools/gpurun_wait.sh <log> <cmd>
LOG=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout 1200 -- "$@" > "$LOG" 2>&1
  rc=$?
  echo "attempt $i rc=$rc" >> "$LOG.attempts"
  if [ $rc -ne 3 ] && ! grep -q '"status": "transient"' gpurun_out/.last_call.json; then exit $rc; fi
  sleep 60
done
exit 3
