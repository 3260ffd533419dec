#!/bin/bash
# Same-box A/B of environment settings on one workload: alternating single-pair bench
# lines (no CPU legs).  usage: env_ab.sh OUTDIR WORKLOAD REPS NAME=ENV[,ENV...] ...
#   e.g. env_ab.sh gpurun_out/ab cal 3 simd=MADPOSE_NOTHING=1 scalar=MADPOSE_SAMPLER_SIMD=0
#   (values that hold commas: separate the settings by '@' instead, e.g. x=A=1,2@B=3)
set -o pipefail
out=$1 wl=$2 reps=$3; shift 3
mkdir -p "$out"
for rep in $(seq 1 "$reps"); do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    if [[ "$envs" == *@* ]]; then sep=${envs//@/ }; else sep=${envs//,/ }; fi
    env $sep timeout -k 10 200 python bench.py --workload "$wl" --cpu-budget 0 --in-flight 1 --steps 40 > "$out/${wl}_${name}_$rep.json" 2>/dev/null || exit $?
    python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["value"]), round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["ms_per_pair"].items()})' "$out/${wl}_${name}_$rep.json" "$wl $name" || exit 1
  done
done
