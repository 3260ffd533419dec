#!/bin/bash
# A/Bs on one box: ScanNet stand-in at the default minimum batch (128) against 512 and
# 1000 (the run's whole iteration budget); cal bench twice (AVX2 inlier compaction in)
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "240:s6/bench_cal_a:python bench.py --cpu-budget 0" \
 "300:s6/scannet_min128:python bench.py --workload scannet --cpu-budget 0" \
 "300:s6/scannet_min512:MADPOSE_MIN_BATCH=512 python bench.py --workload scannet --cpu-budget 0" \
 "300:s6/scannet_min1000:MADPOSE_MIN_BATCH=1000 python bench.py --workload scannet --cpu-budget 0" \
 "240:s6/bench_cal_b:python bench.py --cpu-budget 0"
