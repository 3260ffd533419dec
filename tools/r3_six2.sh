#!/bin/bash
# 6pt deflated-eigen root stage (three kernels): tests, diagnostic, full-size sf, sf
# bench and its kernel statistics
mkdir -p gpurun_out/six2
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300:six2/pytest_uncal:python -u -m pytest tests/test_uncalibrated_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "400:six2/diag:python -u tools/diag_pt67.py 2000 21,23,24,25 ''" \
 "300:six2/fullsize_sf:python -u -m pytest tests/test_full_size_gpu.py -q -k sf --timeout 250 --timeout-method thread" \
 "200:six2/bench_sf:python bench.py --workload sf --cpu-budget 0" \
 "200:six2/prof_sf:rocprofv3 --kernel-trace --stats -d gpurun_out/six2/prof -o sf -- python3 bench.py --workload sf --cpu-budget 0 --in-flight 1 --steps 10 --warmup 2"
