#!/bin/bash
# Record models written by score_batch to mapped host memory (no copy round trip per
# new best): estimator parity tests, cal bench A/B against MADPOSE_FETCH_MODEL=1 on one
# box, then the score_batch PMC passes (tools/r3_s8_pmc.sh)
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "500:s9/pytest_engine:python -u -m pytest tests/test_engine_gpu.py tests/test_full_size_gpu.py tests/test_scannet_gpu.py tests/test_uncalibrated_gpu.py -x -q --timeout 300 --timeout-method thread" \
 "200:s9/bench_cal_rec:python bench.py --cpu-budget 0" \
 "200:s9/bench_cal_copy:MADPOSE_FETCH_MODEL=1 python bench.py --cpu-budget 0" \
 "200:s9/bench_cal_rec2:python bench.py --cpu-budget 0" \
 "200:s9/bench_cal_copy2:MADPOSE_FETCH_MODEL=1 python bench.py --cpu-budget 0" && \
tools/r3_s8_pmc.sh
