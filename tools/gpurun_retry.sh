#!/bin/bash
# Run a gpurun call, retrying ONLY when the harness reports an infrastructure
# event (no box / box lost while preparing / backoff) -- never when the
# command itself ran and failed.  usage: tools/gpurun_retry.sh LOGFILE TIMEOUT CMD...
LOG=$1; shift
TO=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|backing off\|slot(s) on this pod are busy" "$LOG" && ! grep -q "status=ok\|status=fail" "$LOG"; then
    sleep 90
    continue
  fi
  exit $rc
done
exit $rc
