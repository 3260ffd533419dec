#!/bin/bash
# Where score_batch's waves spend their cycles: one rocprofv3 PMC pass (8 SQ counters)
# over a short cal bench; usage: tools/pmc_wait.sh OUTDIR (under gpurun_out/)
export TMPDIR=/tmp
d=${1:-gpurun_out/pmcw}
mkdir -p "$d"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES --output-format csv -d "$d" -o wait -- python3 bench.py --cpu-budget 0 --in-flight 1 --steps 3 --warmup 1 > "$d/wait.log" 2>&1
rc=$?
find "$d" -name '*.csv' | head
exit $rc
