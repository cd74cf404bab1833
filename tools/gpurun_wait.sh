# gpurun with waiting for a free box: re-submits ONLY when gpurun reports that no box / slot was free
# (exit 3, or a "transient" status: nothing ran, nothing was charged); any other outcome ends it.
#   bash tools/gpurun_wait.sh <log> <timeout-s> '<command>'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 60); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  # nothing ran when no box / slot was free, or when this repo's previous call is still running: wait and resubmit
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG" && ! grep -q "already running" "$LOG"; then exit $rc; fi
  sleep 60
done
exit $rc
