#!/bin/bash
# The current tree against an older build in ab_old/ (a git worktree of an earlier
# commit, built in place) on one box: alternating bench lines.  usage: old_ab.sh OUTDIR WORKLOAD...
set -o pipefail
out=${1:-gpurun_out/oldab}; shift
mkdir -p "$out"
for rep in 1 2; do
  for wl in "$@"; do
    if [ "$wl" = scannet ]; then args="--steps 3 --warmup 1 --no-point-only"; else args="--steps 40 --in-flight 1"; fi
    for tree in new old; do
      d=.; [ $tree = old ] && d=ab_old
      (cd $d && timeout -k 10 200 python bench.py --workload $wl --cpu-budget 0 $args) > "$out/${wl}_${tree}_$rep.json" 2>/dev/null || exit $?
      python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["value"],1), round(d["ms_per_step"],3))' "$out/${wl}_${tree}_$rep.json" "$wl $tree" || exit 1
    done
  done
done
