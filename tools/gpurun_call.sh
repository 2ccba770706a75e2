#!/bin/bash
# Local helper (runs in this container, not on the GPU box): one gpurun call.
# Re-submits ONLY when gpurun reports exit 3 ("no box or slot free / box not
# prepared": nothing ran, nothing charged). Any other status is returned as is.
#   usage: tools/gpurun_call.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for attempt in $(seq 1 ${ATTEMPTS:-6}); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  echo "[gpurun_call] attempt $attempt: exit 3 (nothing ran), retrying in ${SLEEP:-60} s" >> "$LOG.retries"
  sleep ${SLEEP:-60}
done
echo "exit $rc" >> "$LOG"
exit $rc
