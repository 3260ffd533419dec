#!/bin/bash
# Short cal bench lines (no CPU legs, one pair in flight) under environment variants:
# usage: tools/cal_ab.sh <outdir> "<label>:<VAR=val ...>" ...   ("-" = no variables)
out=gpurun_out/${1:-calab}; shift
mkdir -p "$out"
wl=${WL:-cal}
for spec in "$@"; do
  label=${spec%%:*}; vars=${spec#*:}; [ "$vars" = "-" ] && vars=""
  env $vars timeout -k 10 150 python bench.py --workload "$wl" --cpu-budget 0 --in-flight 1 --steps ${STEPS:-80} > "$out/$label.json" 2>/dev/null
  rc=$?; [ $rc -ne 0 ] && { echo "$label rc=$rc"; exit $rc; }
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["value"]), round(d["ms_per_step"],3), round(d["speculation"]["solved_over_accepted"],3), {k: round(v,3) for k,v in d["ms_per_pair"].items()})' "$out/$label.json" "$label" || exit 1
done
exit 0
