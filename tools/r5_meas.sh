#!/bin/bash
# Round-5 measurement set: margin/tie/MD/engine GPU tests, the exact-MD stage
# microbenchmark, cal benches with 4 and 2 lanes per MD sample (MADPOSE_MDX_R) under
# rocprofv3 kernel statistics, sf / tf / ScanNet lines, and a cal run with the LO
# phase timers.  Output under gpurun_out/$1 (default r5m).  MADPOSE_R5_TESTS overrides
# the test list ("all" = the whole GPU suite).
out=gpurun_out/${1:-r5m}
mkdir -p "$out"
export TMPDIR=/tmp
step() { # seconds log command...
  local secs=$1 log=$2; shift 2
  echo "== $log"
  timeout -k 10 "$secs" "$@" > "$out/$log" 2>&1
  local rc=$?
  tail -3 "$out/$log"
  case $rc in 0) ;; 1) [ "$log" = pytest.log ] || { echo "fatal rc=1"; exit 1; } ;; *) echo "fatal rc=$rc"; exit $rc ;; esac
  return 0
}
tests=${MADPOSE_R5_TESTS:-"tests/test_margins_gpu.py tests/test_ties_gpu.py tests/test_md_exact_gpu.py tests/test_engine_gpu.py tests/test_full_size_gpu.py tests/test_uncalibrated_gpu.py tests/test_lm_device_gpu.py"}
[ "$tests" = all ] && tests="tests -m gpu"
step 900 pytest.log python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider $tests
step 120 mdx_build.log hipcc -O3 -std=c++17 --offload-arch=gfx950 -I madpose_amd/csrc/include -I include tools/mdx_bench.hip -o tools/mdx_bench
step 60 mdx_bench.log tools/mdx_bench 8192
step 120 mdx_count_build.log hipcc -O3 -std=c++17 -DMDX_COUNT --offload-arch=gfx950 -I madpose_amd/csrc/include -I include tools/mdx_bench.hip -o tools/mdx_count
step 60 mdx_count.log tools/mdx_count 32768
step 120 score_build.log hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I madpose_amd/csrc/include tools/score_bench.hip -o tools/score_bench
step 60 score_bench.log tools/score_bench 8192 0
step 240 bench_cal.log python -u bench.py --cpu-budget 0
step 240 prof_cal4.log rocprofv3 --kernel-trace --stats -d "$out/prof_cal4" -o cal -- python3 bench.py --cpu-budget 0 --in-flight 1
step 60 cal4_summary.log python tools/prof_summary.py "$out/prof_cal4" "$out/cal4_kernel_stats.csv"
MADPOSE_MDX_R=2 step 240 bench_cal_r2.log python -u bench.py --cpu-budget 0
step 200 bench_sf.log python -u bench.py --workload sf --cpu-budget 0
step 200 bench_tf.log python -u bench.py --workload tf --cpu-budget 0
step 200 bench_scannet.log python -u bench.py --workload scannet --cpu-budget 0
MADPOSE_LO_TIMING=1 step 240 bench_cal_lot.log python -u bench.py --cpu-budget 0
# same-box A/B of environment settings: MADPOSE_R5_AB="NAME=VAL ..." (space separated;
# each run alternates the default and every setting, MADPOSE_R5_REPS times)
if [ -n "$MADPOSE_R5_AB" ]; then
  for rep in $(seq 1 ${MADPOSE_R5_REPS:-2}); do
    step 200 ab_default_$rep.log python -u bench.py --cpu-budget 0
    for kv in $MADPOSE_R5_AB; do
      k=${kv%%=*}; v=${kv#*=}
      export "$kv"; step 200 ab_${k}_${v}_$rep.log python -u bench.py --cpu-budget 0; unset "$k"
    done
  done
fi
exit 0
