#!/bin/bash
# PMC passes of score_batch on the current kernel (exact early exit + record skip), one
# counter group per run as the MI355X guide prescribes, then the per-iteration fit that
# bench.py reads (profiles/r03/pmc_score_batch.json, written on the build host)
export TMPDIR=/tmp
mkdir -p gpurun_out/s8
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d gpurun_out/s8 -o sq -- python3 bench.py --cpu-budget 0 --in-flight 1 --steps 3 --warmup 1 > gpurun_out/s8/sq.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/s8 -o fetch -- python3 bench.py --cpu-budget 0 --in-flight 1 --steps 3 --warmup 1 > gpurun_out/s8/fetch.log 2>&1
rc=$?
ls gpurun_out/s8
exit $rc
