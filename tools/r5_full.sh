#!/bin/bash
# Round-5 measurement set on the current tree: the GPU suite, smoke(), the default bench
# line (cal, CPU baselines), sf / tf / ScanNet lines, rocprofv3 kernel statistics of
# short cal, sf and tf runs, a cal run with the LO phase timers and a cal timeline.
# Output under gpurun_out/$1 (default r5f).  MADPOSE_R5_SKIP_TESTS=1 skips the suite.
out=gpurun_out/${1:-r5f}
mkdir -p "$out"
export TMPDIR=/tmp
step() { # seconds log command...
  local secs=$1 log=$2; shift 2
  echo "== $log"
  timeout -k 10 "$secs" "$@" > "$out/$log" 2>&1
  local rc=$?
  tail -2 "$out/$log" | cut -c1-300
  case $rc in 0) ;; 1) [ "$log" = pytest_gpu.log ] || { echo "fatal rc=1"; exit 1; } ;; *) echo "fatal rc=$rc"; exit $rc ;; esac
  return 0
}
[ -n "$MADPOSE_R5_SKIP_TESTS" ] || step 700 pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
step 200 smoke.log python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step 300 bench_cal.log python -u bench.py
step 200 bench_sf.log python -u bench.py --workload sf --cpu-budget 0
step 200 bench_tf.log python -u bench.py --workload tf --cpu-budget 0
step 200 bench_scannet.log python -u bench.py --workload scannet --cpu-budget 0
step 240 prof_cal.log rocprofv3 --kernel-trace --stats -d "$out/prof_cal" -o cal -- python3 bench.py --cpu-budget 0 --in-flight 1
step 60 cal_summary.log python tools/prof_summary.py "$out/prof_cal" "$out/cal_kernel_stats.csv"
step 240 prof_sf.log rocprofv3 --kernel-trace --stats -d "$out/prof_sf" -o sf -- python3 bench.py --workload sf --cpu-budget 0 --in-flight 1
step 60 sf_summary.log python tools/prof_summary.py "$out/prof_sf" "$out/sf_kernel_stats.csv"
step 240 prof_tf.log rocprofv3 --kernel-trace --stats -d "$out/prof_tf" -o tf -- python3 bench.py --workload tf --cpu-budget 0 --in-flight 1
step 60 tf_summary.log python tools/prof_summary.py "$out/prof_tf" "$out/tf_kernel_stats.csv"
MADPOSE_LO_TIMING=1 step 200 bench_cal_lot.log python -u bench.py --cpu-budget 0 --in-flight 1
MADPOSE_TIMELINE=20-22 step 200 timeline.log python -u bench.py --cpu-budget 0 --in-flight 1
exit 0
