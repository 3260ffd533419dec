#!/bin/bash
# The 15 x 15 lockstep QR (eig15_gen.h) after a generator change: root-stage timings
# and bit-identity against the 16-lane group QR (tools/eig6_bench), the 6pt parity
# tests, then sf bench lines and a kernel-trace profile.  usage: eig_ab.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/eig}
mkdir -p "$out"
for ns in 512 2048 8192; do
  timeout -k 10 120 tools/eig6_bench $ns > "$out/eig_$ns.log" 2>&1 || exit $?
done
grep -h "samples\|group QR\|lockstep QR" "$out"/eig_*.log
timeout -k 10 600 python -u -m pytest tests/test_uncalibrated_gpu.py tests/test_sixpt_hard.py tests/test_full_size_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/pytest.log" 2>&1; rc=$?; tail -n 3 "$out/pytest.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 120 python bench.py --workload sf --cpu-budget 0 --in-flight 1 --steps 40 > "$out/sf_$r.json" 2>/dev/null || exit $?
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print("sf", round(d["value"]), round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["ms_per_pair"].items()})' "$out/sf_$r.json" || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$out/prof_sf" -o sf -- python bench.py --workload sf --cpu-budget 0 --in-flight 1 --steps 20 > "$out/prof_sf.log" 2>&1 || exit $?
python tools/prof_summary.py "$out/prof_sf" "$out/sf_kernel_stats.csv" > "$out/sf_kernel_summary.txt"
head -n 12 "$out/sf_kernel_summary.txt"
