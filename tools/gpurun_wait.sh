# Run one gpurun command, retrying only while the pool has no free slot or box (a "transient"
# verdict in gpurun_out/.last_call.json: nothing ran, nothing charged); any other outcome ends
# it (the command's own exit codes may overlap gpurun's).  Usage: bash tools/gpurun_wait.sh <log> <cmd>
LOG=$1; shift
for i in $(seq 1 30); do
  rm -f gpurun_out/.last_call.json
  /usr/local/graft/bin/gpurun --timeout 1200 -- "$@" > "$LOG" 2>&1
  rc=$?
  echo "attempt $i rc=$rc" >> "$LOG.attempts"
  { grep -q '"status": "transient"' gpurun_out/.last_call.json 2>/dev/null || grep -q 'status=transient' "$LOG"; } || exit $rc
  sleep 60
done
exit 3
