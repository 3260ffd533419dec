#!/bin/bash
# Same-box A/B of environment settings on the ScanNet stand-in (pairs/s, no CPU legs).
# usage: sn_ab.sh OUTDIR REPS NAME=ENV[,ENV...] ...
set -o pipefail
out=$1 reps=$2; shift 2
mkdir -p "$out"
for rep in $(seq 1 "$reps"); do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    env ${envs//,/ } timeout -k 10 200 python bench.py --workload scannet --cpu-budget 0 --steps ${SN_STEPS:-5} --warmup 1 > "$out/sn_${name}_$rep.json" 2>/dev/null || exit $?
    python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["value"], 1), d["pose_auc"]["5"])' "$out/sn_${name}_$rep.json" "$name" || exit 1
  done
done
