#!/bin/bash
# Run one gpurun call, waiting for a free GPU slot: re-issues the SAME call only while gpurun
# reports that no slot / box was free (nothing ran, nothing charged); any call that ran ends it.
# usage: tools/gpurun_wait.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 20); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUT 2>&1
  rc=$?
  if grep -q "nothing was charged\|stopped responding while being prepared\|backing off\|no free box" $OUT && ! grep -q "status=ok\|status=fail" $OUT; then
    sleep 120
    continue
  fi
  exit $rc
done
exit 3
