#!/bin/bash
# Local helper: re-submit a gpurun call ONLY when the infrastructure reports "no box / transient" (exit 3,
# nothing ran, nothing charged).  Any other exit code (including GPU failures) is returned as is.
# Usage: scripts/gpurun_retry.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUT 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then exit $rc; fi
  grep -q "status=transient\|no box\|slot" $OUT || exit $rc
  sleep $((20 * i))
done
exit 3
