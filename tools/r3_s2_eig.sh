#!/bin/bash
# Shared-focal root stage after the LDS trim of the deflation kernel and the
# samples-per-wave packing of the lockstep QR: kernel timings at 2048 / 16384 samples,
# the 6pt / LM GPU tests, full-size sf parity, sf bench with rocprof statistics
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "60:s2e/eig_2048:tools/eig6_bench 2048" \
 "90:s2e/eig_16384:tools/eig6_bench 16384" \
 "400:s2e/pytest_six:python -u -m pytest tests/test_uncalibrated_gpu.py tests/test_sixpt_hard.py tests/test_lm_device_gpu.py -x -q --timeout 200 --timeout-method thread" \
 "300:s2e/fullsize_sf:python -u -m pytest tests/test_full_size_gpu.py -q -k sf --timeout 250 --timeout-method thread" \
 "240:s2e/prof_sf:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s2e/prof -o sf -- python3 bench.py --workload sf --cpu-budget 0 --in-flight 1 --steps 10 --warmup 2"
