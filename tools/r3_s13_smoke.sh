#!/bin/bash
# smoke() on the final tree and the tf kernel statistics
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300:s13/smoke:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "200:s13/prof_tf:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s13/prof -o tf -- python3 bench.py --workload tf --cpu-budget 0 --in-flight 1 --steps 10 --warmup 2"
