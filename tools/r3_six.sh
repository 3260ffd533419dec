#!/bin/bash
# 6pt deflated-eigen root stage: unit tests, the 2000-trial device-vs-oracle diagnostic
# on four seeds, full-size sf parity, sf bench (eig vs the old DFT kernel).
mkdir -p gpurun_out/six
tools/gpu_steps.sh \
 "300:six/pytest_uncal:python -u -m pytest tests/test_uncalibrated_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "400:six/diag:python -u tools/diag_pt67.py 2000 21,23,24,25 ''" \
 "300:six/fullsize_sf:python -u -m pytest tests/test_full_size_gpu.py -q -k sf --timeout 250 --timeout-method thread" \
 "200:six/bench_sf_eig:python bench.py --workload sf --cpu-budget 0" \
 "200:six/bench_sf_dft:MADPOSE_PT6_DFT=1 python bench.py --workload sf --cpu-budget 0"
