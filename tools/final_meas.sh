# Round-end measurement set: default bench line (with CPU baselines), rocprofv3 kernel
# statistics of the same command (short run), sf / tf lines.
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 240 python bench.py > gpurun_out/final/bench_cal_default.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o cal -- python3 bench.py --cpu-budget 0 --in-flight 1 > gpurun_out/final/bench_cal_under_rocprof.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --workload sf --cpu-budget 0 > gpurun_out/final/bench_sf.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --workload tf --cpu-budget 0 > gpurun_out/final/bench_tf.log 2>&1 || exit $?
find gpurun_out/final -name '*stats*'
