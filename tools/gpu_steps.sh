#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that
# ends in a fault/abort/segfault/timeout (non-fatal test failures continue).
# usage: tools/gpu_steps.sh "<seconds>:<logname>:<command>" ...
mkdir -p gpurun_out
worst=0
for spec in "$@"; do
  secs=${spec%%:*}; rest=${spec#*:}; log=${rest%%:*}; cmd=${rest#*:}
  mkdir -p "gpurun_out/$(dirname "$log")"
  echo "== step $log ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$log.log" 2>&1
  rc=$?
  echo "== step $log rc=$rc"
  tail -5 "gpurun_out/$log.log"
  case $rc in
    0) ;;
    124|134|137|139|250|251|245) echo "fatal rc=$rc, stopping"; exit $rc ;;
    *) worst=$rc ;;
  esac
done
exit $worst
