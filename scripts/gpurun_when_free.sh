#!/bin/bash
# Submit one gpurun call, re-submitting it only while the pool has no box or slot for it (gpurun exit 3 /
# a "transient" verdict with nothing run and nothing charged). A call that ran — whatever its result —
# is never repeated. Usage: scripts/gpurun_when_free.sh LOG TIMEOUT 'command'
log=$1
to=$2
cmd=$3
for attempt in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient rc=None charged=0.0s\|status=transient rc=None charged=Nones" "$log"; then
    echo "[when_free] attempt $attempt: no box (rc=$rc); waiting" >> "$log.attempts"
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
