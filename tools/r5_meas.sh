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
step 240 bench_cal.log python -u bench.py --cpu-budget 0
step 240 prof_cal4.log rocprofv3 --kernel-trace --stats -d "$out/prof_cal4" -o cal -- python3 bench.py --cpu-budget 0 --in-flight 1
step 60 cal4_summary.log python tools/prof_summary.py "$out/prof_cal4" "$out/cal4_kernel_stats.csv"
MADPOSE_MDX_R=2 step 240 bench_cal_r2.log python -u bench.py --cpu-budget 0
step 200 bench_sf.log python -u bench.py --workload sf --cpu-budget 0
step 200 bench_tf.log python -u bench.py --workload tf --cpu-budget 0
step 200 bench_scannet.log python -u bench.py --workload scannet --cpu-budget 0
MADPOSE_LO_TIMING=1 step 240 bench_cal_lot.log python -u bench.py --cpu-budget 0
exit 0
