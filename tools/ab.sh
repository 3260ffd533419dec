#!/bin/bash
# Same-box A/B of environment settings on the bench:
#   tools/ab.sh OUT REPS "BENCH ARGS" SETTING...
# SETTING: "default" or space-separated NAME=VAL pairs (one quoted word per setting).
# Each rep runs every setting once, in order; logs gpurun_out/OUT/ab_<i>_<rep>.log.
out=gpurun_out/$1; reps=$2; args=$3; shift 3
mkdir -p "$out"
for rep in $(seq 1 "$reps"); do
  i=0
  for set in "$@"; do
    i=$((i + 1))
    log="$out/ab_${i}_$rep.log"
    echo "== $set (rep $rep)" | tee "$log"
    (
      [ "$set" = default ] || for kv in $set; do export "$kv"; done
      timeout -k 10 200 python -u bench.py $args >> "$log" 2>&1
    )
    rc=$?
    tail -1 "$log" | cut -c1-200
    [ $rc -eq 0 ] || { echo "fatal rc=$rc"; exit $rc; }
  done
done
exit 0
