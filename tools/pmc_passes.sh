#!/bin/bash
# PMC passes of score_batch for the roofline fit (tools/pmc_score.py), one counter group
# per rocprofv3 run as the MI355X guide prescribes; usage: tools/pmc_passes.sh OUTDIR
# (under gpurun_out/), run on the GPU box.
export TMPDIR=/tmp
d=${1:-gpurun_out/pmc}
mkdir -p "$d"
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d "$d" -o sq -- python3 bench.py --cpu-budget 0 --in-flight 1 --steps 3 --warmup 1 > "$d/sq.log" 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$d" -o fetch -- python3 bench.py --cpu-budget 0 --in-flight 1 --steps 3 --warmup 1 > "$d/fetch.log" 2>&1
rc=$?
find "$d" -name '*.csv' | head
exit $rc
