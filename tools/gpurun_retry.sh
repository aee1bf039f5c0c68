#!/bin/bash
# usage: tools/gpurun_retry.sh TIMEOUT OUTFILE 'command'
# Retries gpurun only on infrastructure-transient outcomes (never on a failing command).
T=$1; OUT=$2; CMD=$3
for i in 1 2 3 4 5; do
  /usr/local/graft/bin/gpurun --timeout $T -- "$CMD" > $OUT 2>&1
  rc=$?
  if grep -q "status=transient\|rc=3\b\|no box or slot" $OUT || [ $rc -eq 3 ]; then sleep 60; continue; fi
  break
done
tail -3 $OUT
