#!/bin/bash
# rocprofv3 kernel statistics of a short bench run: tools/prof_wl.sh <workload> <outdir>
wl=${1:-cal}; out=gpurun_out/${2:-prof_$wl}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$out/prof" -o "$wl" -- python3 bench.py --workload "$wl" --cpu-budget 0 --in-flight 1 --steps ${STEPS:-20} > "$out/prof.log" 2>&1 || exit $?
python tools/prof_summary.py "$out/prof" "$out/${wl}_kernel_stats.csv"
