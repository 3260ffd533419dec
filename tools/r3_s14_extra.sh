#!/bin/bash
# Final-tree extras: the LO phase breakdown on cal (MADPOSE_LO_TIMING=1, stderr), and the
# two-rank rehearsal of the N>1 path on the one card (gloo, both ranks on device 0)
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "200:s14/bench_cal_lo_timing:MADPOSE_LO_TIMING=1 python bench.py --cpu-budget 0 --steps 20 --warmup 2" \
 "300:s14/bench_two_ranks:MADPOSE_BENCH_DIST_BACKEND=gloo MADPOSE_BENCH_DEVICE=0 python bench.py --gpus 2 --cpu-budget 0 --steps 20 --warmup 2"
