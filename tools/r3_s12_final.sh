#!/bin/bash
# Final round-3 measurement set (after the tail / check-schedule changes): full GPU suite, default bench lines (cal with the CPU
# baseline, sf, tf, ScanNet stand-in), rocprofv3 kernel statistics of cal and sf
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "900:s12/pytest_gpu:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
 "240:s12/bench_cal:python bench.py" \
 "200:s12/bench_sf:python bench.py --workload sf --cpu-budget 0" \
 "200:s12/bench_tf:python bench.py --workload tf --cpu-budget 0" \
 "300:s12/bench_scannet:python bench.py --workload scannet --cpu-budget 0" \
 "200:s12/prof_cal:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s12/prof -o cal -- python3 bench.py --cpu-budget 0 --in-flight 1 --steps 10 --warmup 2" \
 "200:s12/prof_sf:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s12/prof -o sf -- python3 bench.py --workload sf --cpu-budget 0 --in-flight 1 --steps 10 --warmup 2"
