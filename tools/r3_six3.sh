#!/bin/bash
# 6pt lockstep-QR root stage: kernel timings, unit tests, the 2000-trial device-vs-oracle
# diagnostic on four seeds, full-size sf parity, sf bench (lockstep vs wave hqr vs DFT)
mkdir -p gpurun_out/six3
tools/gpu_steps.sh \
 "60:six3/eig_2048:tools/eig6_bench 2048" \
 "60:six3/eig_64:tools/eig6_bench 64" \
 "300:six3/pytest_uncal:python -u -m pytest tests/test_uncalibrated_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "400:six3/diag:python -u tools/diag_pt67.py 2000 21,23,24,25 ''" \
 "300:six3/fullsize_sf:python -u -m pytest tests/test_full_size_gpu.py -q -k sf --timeout 250 --timeout-method thread" \
 "200:six3/bench_sf:python bench.py --workload sf --cpu-budget 0 --in-flight 1" \
 "200:six3/bench_sf_dft:MADPOSE_PT6_DFT=1 python bench.py --workload sf --cpu-budget 0 --in-flight 1"
