#!/bin/bash
# Round-3 measurement set on the current tree: full GPU suite, the default bench lines
# (cal with the CPU baseline, sf, tf, ScanNet stand-in) and the cal / sf / tf kernel
# statistics (rocprofv3 kernel trace, CSV)
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "900:s3/pytest_gpu:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "240:s3/bench_cal:python bench.py" \
 "200:s3/bench_sf:python bench.py --workload sf --cpu-budget 0" \
 "200:s3/bench_tf:python bench.py --workload tf --cpu-budget 0" \
 "300:s3/bench_scannet:python bench.py --workload scannet --cpu-budget 0" \
 "200:s3/prof_cal:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s3/prof -o cal -- python3 bench.py --cpu-budget 0 --in-flight 1 --steps 10 --warmup 2" \
 "200:s3/prof_tf:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s3/prof -o tf -- python3 bench.py --workload tf --cpu-budget 0 --in-flight 1 --steps 10 --warmup 2"
