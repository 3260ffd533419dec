#!/bin/bash
# 16-lane group deflation (+ balance + Hessenberg): timings and root agreement against
# the one-wave kernel at 512 / 2048 / 16384 samples, the 6pt GPU tests, full-size sf
# parity, sf and ScanNet stand-in bench lines with the group deflation as default
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "60:s5/eig_512:tools/eig6_bench 512" \
 "60:s5/eig_2048:tools/eig6_bench 2048" \
 "90:s5/eig_16384:tools/eig6_bench 16384" \
 "400:s5/pytest_six:python -u -m pytest tests/test_uncalibrated_gpu.py tests/test_sixpt_hard.py tests/test_engine_gpu.py tests/test_scannet_gpu.py -x -q --timeout 250 --timeout-method thread" \
 "300:s5/fullsize_sf:python -u -m pytest tests/test_full_size_gpu.py -q -k sf --timeout 250 --timeout-method thread" \
 "200:s5/bench_sf:python bench.py --workload sf --cpu-budget 0" \
 "300:s5/bench_scannet:python bench.py --workload scannet --cpu-budget 0"
