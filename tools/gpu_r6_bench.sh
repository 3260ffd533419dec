# Bench lines of the four workloads into gpurun_out/$1/ (run from the repo root on the box).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/$1; mkdir -p $D
shift
for wl in ${WLS:-cal sf tf scannet}; do
  timeout -k 10 400 python -u bench.py --workload $wl ${BENCH_ARGS:-} > $D/bench_$wl.log 2>&1 || exit $?
  tail -1 $D/bench_$wl.log | cut -c1-300
done
