set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6a
timeout -k 10 900 python -u -m pytest tests/test_teardown_gpu.py tests/test_switch_invariance_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6a/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r6a/pytest.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
MADPOSE_SEGV_MAPS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r6a/prof_sn -o sn -- python3 $GRAFT_REPO_ROOT/bench.py --workload scannet --cpu-budget 0 --steps 3 --warmup 1 --no-point-only > $GRAFT_REPO_ROOT/gpurun_out/r6a/prof_sn.log 2>&1
echo "rocprof rc=$?"
tail -2 $GRAFT_REPO_ROOT/gpurun_out/r6a/prof_sn.log
