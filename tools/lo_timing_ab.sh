#!/bin/bash
# LO phase times (MADPOSE_LO_TIMING) of a bench workload (WL, default cal) under
# environment variants: the per-LO averages of the engine's timing lines, averaged over
# the timed pairs.  usage: [WL=tf] lo_timing_ab.sh OUTDIR REPS NAME=ENV[,ENV...] ...
set -o pipefail
out=$1 reps=$2; shift 2
mkdir -p "$out"
for rep in $(seq 1 "$reps"); do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    env MADPOSE_LO_TIMING=1 ${envs//,/ } timeout -k 10 200 python bench.py --workload "${WL:-cal}" --cpu-budget 0 --in-flight 1 --steps 40 > "$out/${WL:-cal}_${name}_$rep.json" 2> "$out/${WL:-cal}_${name}_$rep.err" || exit $?
    python - "$out/${WL:-cal}_${name}_$rep" "$name" <<'PY' || exit 1
import json, re, sys
base, name = sys.argv[1], sys.argv[2]
d = json.loads(open(base + ".json").read().strip().splitlines()[-1])
keys = ["prefix", "steps", "step0", "step0 fit", "step0 lsq", "step0 iters", "before the parallel run", "the run", "the speculation hook"]
acc = {k: [] for k in keys}
for line in open(base + ".err"):
    if " LO: " not in line and "LO steps phase" not in line:
        continue
    for k in keys:
        m = re.search(re.escape(k) + r" ([0-9.]+) us", line)
        if m:
            acc[k].append(float(m.group(1)))
print(name, round(d["ms_per_step"], 3), {k: round(sum(v) / len(v), 1) for k, v in acc.items() if v})
PY
  done
done
