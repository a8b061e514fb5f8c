#!/bin/bash
# gpurun with retries ONLY when no box is free (rc 3: nothing ran, nothing charged)
# usage: gpr.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; shift 2
for i in $(seq 1 30); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "no free box right now" $LOG; then echo "rc=$rc" >> $LOG; exit $rc; fi
  sleep 60
done
