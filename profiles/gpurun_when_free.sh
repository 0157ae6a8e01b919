#!/bin/bash
# Run one gpurun call, re-submitting it only while gpurun answers 3 ("no box or
# slot free right now": nothing ran, nothing was charged), at most N tries,
# WAIT seconds apart.  Any other exit status ends it (a refusal, a failure or
# a finished run is never resubmitted).
#   bash profiles/gpurun_when_free.sh OUT N WAIT TIMEOUT 'command'
OUT=$1; N=$2; WAIT=$3; TO=$4; CMD=$5
for i in $(seq 1 $N); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > "$OUT" 2>&1
  rc=$?
  echo "[try $i rc=$rc $(date +%T)]" >> "$OUT.tries"
  [ $rc -ne 3 ] && exit $rc
  sleep $WAIT
done
exit 3
