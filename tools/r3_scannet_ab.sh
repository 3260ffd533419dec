#!/bin/bash
# ScanNet stand-in A/B: root stage (eig vs DFT), batch growth, pairs in flight
mkdir -p gpurun_out/sab
tools/gpu_steps.sh \
 "200:sab/default:python bench.py --workload scannet --cpu-budget 0 --no-point-only" \
 "200:sab/dft:MADPOSE_PT6_DFT=1 python bench.py --workload scannet --cpu-budget 0 --no-point-only" \
 "200:sab/g4:MADPOSE_BATCH_GROWTH=4 python bench.py --workload scannet --cpu-budget 0 --no-point-only" \
 "200:sab/dft_g4:MADPOSE_PT6_DFT=1 MADPOSE_BATCH_GROWTH=4 python bench.py --workload scannet --cpu-budget 0 --no-point-only" \
 "200:sab/s16:python bench.py --workload scannet --cpu-budget 0 --no-point-only --streams 16" \
 "200:sab/s16_g4:MADPOSE_BATCH_GROWTH=4 python bench.py --workload scannet --cpu-budget 0 --no-point-only --streams 16" \
 "400:sab/pytest_lm:python -u -m pytest tests/test_lm_device_gpu.py tests/test_sixpt_hard.py tests/test_uncalibrated_gpu.py -x -q --timeout 300 --timeout-method thread"
