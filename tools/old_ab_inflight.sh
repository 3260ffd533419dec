#!/bin/bash
# The current tree against the ab_old/ build on one box, cal bench with its 8-pairs-in-
# flight leg.  usage: old_ab_inflight.sh OUTDIR REPS
set -o pipefail
out=${1:-gpurun_out/oldabif}; reps=${2:-2}
mkdir -p "$out"
for rep in $(seq 1 "$reps"); do
  for tree in new old; do
    d=.; [ $tree = old ] && d=ab_old
    (cd $d && timeout -k 10 200 python bench.py --cpu-budget 0 --steps 40) > "$out/cal_${tree}_$rep.json" 2>/dev/null || exit $?
    python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); f=d["pairs_in_flight"]; print(sys.argv[2], round(d["value"]), round(d["ms_per_step"],3), "in flight", round(f["hypotheses_per_s"]), round(f["ms_per_pair"],3))' "$out/cal_${tree}_$rep.json" "cal $tree" || exit 1
  done
done
