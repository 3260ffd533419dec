#!/bin/bash
# Lanes per shared-focal sample of the exact MD kernel (MADPOSE_MDX_R = 1 / 2 / 4 / 8):
# sf bench lines (no CPU legs) alternating the settings, then a kernel-trace profile of
# each.  usage: mdxr_ab.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/mdxr}
mkdir -p "$out"
for rep in 1 2; do
  for r in 1 2 4 8; do
    MADPOSE_MDX_R=$r timeout -k 10 120 python bench.py --workload sf --cpu-budget 0 --in-flight 1 --steps 40 > "$out/sf_r${r}_$rep.json" 2>/dev/null || exit $?
    python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["value"]), round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["ms_per_pair"].items()})' "$out/sf_r${r}_$rep.json" "R=$r" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2 4 8; do
  MADPOSE_MDX_R=$r timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$out/prof_r$r" -o sf -- python bench.py --workload sf --cpu-budget 0 --in-flight 1 --steps 20 > "$out/prof_r$r.log" 2>&1 || exit $?
  python tools/prof_summary.py "$out/prof_r$r" "$out/sf_r${r}_kernel_stats.csv" > "$out/sf_r${r}_kernel_summary.txt"
  echo "R=$r"; head -n 4 "$out/sf_r${r}_kernel_summary.txt" | cut -c1-140
done
