#!/bin/bash
# Early-exit check schedule A/B (MADPOSE_SCORE_CHECK="first,every" in trips of 256
# correspondences) after the DPP wave sum; GPU suite first.
tools/gpu_steps.sh \
 "400:pytest_gpu:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "200:cal_default:python bench.py --cpu-budget 0" \
 "200:cal_c11:MADPOSE_SCORE_CHECK=1,1 python bench.py --cpu-budget 0" \
 "200:cal_c22:MADPOSE_SCORE_CHECK=2,2 python bench.py --cpu-budget 0" \
 "200:cal_c31:MADPOSE_SCORE_CHECK=3,1 python bench.py --cpu-budget 0" \
 "200:cal_noexit:MADPOSE_SCORE_EXIT=0 python bench.py --cpu-budget 0" \
 "200:sf_default:python bench.py --workload sf --cpu-budget 0" \
 "200:sf_c11:MADPOSE_SCORE_CHECK=1,1 python bench.py --workload sf --cpu-budget 0" \
 "200:tf_default:python bench.py --workload tf --cpu-budget 0" \
 "200:tf_c22:MADPOSE_SCORE_CHECK=2,2 python bench.py --workload tf --cpu-budget 0"
