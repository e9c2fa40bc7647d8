#!/bin/bash
# Re-issue a gpurun call while the pool has no free box (exit 3: nothing ran,
# nothing charged); any other outcome ends the loop.  usage: gpu_retry.sh <log> <timeout> <cmd>
LOG=$1; TO=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 60
done
exit 3
