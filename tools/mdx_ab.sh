#!/bin/bash
# A/B of the exact MD kernel's samples per wave (MADPOSE_MDX_SPW) on sf / tf, short
# bench lines (no CPU legs), then a kernel-trace profile of the default on sf.
set -o pipefail
mkdir -p gpurun_out/mdx
timeout -k 10 300 python -u -m pytest tests/test_md_exact_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mdx/pytest_mdx.log 2>&1; tail -3 gpurun_out/mdx/pytest_mdx.log
for wl in sf tf; do
  for spw in 64 16 8 4; do
    MADPOSE_MDX_SPW=$spw timeout -k 10 120 python bench.py --workload $wl --cpu-budget 0 --in-flight 1 --steps 40 > gpurun_out/mdx/${wl}_${spw}.json 2>/dev/null || exit $?
    python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["value"]), round(d["ms_per_step"],3), round(d["roofline"]["solve_ms_per_launch"],3), {k: round(v,3) for k,v in d["ms_per_pair"].items()})' gpurun_out/mdx/${wl}_${spw}.json "$wl spw=$spw" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/mdx/prof_sf -o sf -- python bench.py --workload sf --cpu-budget 0 --in-flight 1 --steps 20 > gpurun_out/mdx/prof_sf.log 2>&1 || exit $?
python tools/prof_summary.py gpurun_out/mdx/prof_sf gpurun_out/mdx/sf_kernel_stats.csv > gpurun_out/mdx/sf_kernel_summary.txt
cat gpurun_out/mdx/sf_kernel_summary.txt
