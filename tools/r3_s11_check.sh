#!/bin/bash
# score_batch early-exit check schedule (MADPOSE_SCORE_CHECK=first,every in trips of
# 256 correspondences; default N/4, N/4 = 2,2 at N = 2000 and 4,4 at N = 4000): the
# HIP-event launch average of each setting, cal / sf / tf, one box
export TMPDIR=/tmp
steps=""
for cfg in "cal:" "cal:MADPOSE_SCORE_CHECK=1,1" "cal:MADPOSE_SCORE_CHECK=1,2" "cal:MADPOSE_SCORE_CHECK=3,3" \
           "sf:" "sf:MADPOSE_SCORE_CHECK=1,1" "sf:MADPOSE_SCORE_CHECK=1,2" \
           "tf:" "tf:MADPOSE_SCORE_CHECK=2,2" "tf:MADPOSE_SCORE_CHECK=2,4"; do
  wl=${cfg%%:*}; env=${cfg#*:}
  tag=$(echo "${wl}_${env:-default}" | tr '=,' '__')
  steps="$steps \"150:s11/$tag:$env python bench.py --workload $wl --cpu-budget 0 --steps 20 --warmup 2\""
done
eval tools/gpu_steps.sh $steps
