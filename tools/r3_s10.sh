#!/bin/bash
# Record skip decided at the early-exit checks (no entry barrier) and the generated QR's
# single reflector division: lane/group QR bit-identity, estimator parity tests (ScanNet
# all 1500 pairs), cal bench twice, then the score_batch PMC passes
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "60:s10/eig_2048:tools/eig6_bench 2048" \
 "600:s10/pytest_engine:python -u -m pytest tests/test_engine_gpu.py tests/test_full_size_gpu.py tests/test_scannet_gpu.py tests/test_uncalibrated_gpu.py tests/test_sixpt_hard.py -x -q --timeout 400 --timeout-method thread" \
 "200:s10/bench_cal:python bench.py --cpu-budget 0" \
 "200:s10/bench_cal2:python bench.py --cpu-budget 0" && \
sed 's#gpurun_out/s8#gpurun_out/s10p#g' tools/r3_s8_pmc.sh > /tmp/pmc10.sh && bash /tmp/pmc10.sh
