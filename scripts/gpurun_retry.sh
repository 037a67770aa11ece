#!/bin/bash
# Run one gpurun call, retrying ONLY when gpurun itself reports an infrastructure condition
# (exit 3: no box / box lost while being prepared — nothing ran, nothing charged). Any other exit
# status, including a failing GPU command, is returned as is.
# usage: scripts/gpurun_retry.sh <log> <timeout-seconds> '<command>'
log=$1; to=$2; cmd=$3
for i in $(seq 1 ${RETRIES:-8}); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  grep -q "transient\|backing off\|stopped responding\|taken away\|no box" "$log" || break
  sleep ${RETRY_SLEEP:-150}
done
exit $rc
