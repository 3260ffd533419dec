#!/bin/bash
# Full GPU suite, the default bench lines (cal with the CPU baseline, sf, tf, scannet)
# and the cal kernel statistics (rocprofv3, CSV)
mkdir -p gpurun_out/full
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "900:full/pytest_gpu:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "240:full/bench_cal:python bench.py" \
 "200:full/bench_sf:python bench.py --workload sf --cpu-budget 0" \
 "200:full/bench_tf:python bench.py --workload tf --cpu-budget 0" \
 "300:full/bench_scannet:python bench.py --workload scannet --cpu-budget 0" \
 "200:full/prof_cal:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/full/prof -o cal -- python3 bench.py --cpu-budget 0 --in-flight 1 --steps 10 --warmup 2"
