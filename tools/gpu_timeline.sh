set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/t1; mkdir -p $D
for wl in cal sf; do
  MADPOSE_TIMELINE=20-22 timeout -k 10 200 python -u bench.py --workload $wl --cpu-budget 0 --in-flight 1 --steps 20 --prof-every 1 > $D/$wl.log 2> $D/${wl}_tl.log || exit $?
  python tools/timeline_summary.py $D/${wl}_tl.log > $D/${wl}_tl_summary.txt || exit $?
  tail -1 $D/$wl.log | cut -c1-400
done
