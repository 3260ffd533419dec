#!/bin/bash
# Run one gpurun call, retrying only while no box or slot is free (exit 3: nothing ran,
# nothing charged).  usage: tools/gpurun_retry.sh <log> <timeout> <command>
log=$1; to=$2; shift 2
for a in 1 2 3 4 5 6 7 8 9 10 11 12; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  echo "rc=$rc attempt=$a" >> "$log"
  [ $rc -ne 3 ] && exit $rc
  sleep 120
done
exit 3
