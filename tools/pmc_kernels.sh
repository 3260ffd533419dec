#!/bin/bash
# Per-kernel PMC passes of one bench workload (the solver chain's
# figures), one counter group per rocprofv3 run as the MI355X guide prescribes.
# usage (repo root on the box): bash tools/pmc_kernels.sh <dir> <workload> [bench args]
# writes gpurun_out/<dir>/pmc_<workload>_{issue,wait,fetch}/ and <workload>_pmc.txt
# (tools/pmc_kernels.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/$1; W=$2; shift 2
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
run() {  # run <name> <counters...>
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $D/pmc_${W}_$n -o $n -- \
    python3 $R/bench.py --workload $W --cpu-budget 0 --in-flight 1 --steps 3 --warmup 1 "${BENCH_EXTRA[@]}" \
    > $D/pmc_${W}_$n.log 2>&1
}
BENCH_EXTRA=("$@")
run issue SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 && \
run wait SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT && \
run fetch FETCH_SIZE GRBM_GUI_ACTIVE || exit $?
cd $R && python3 tools/pmc_kernels.py $D/pmc_${W}_issue $D/pmc_${W}_wait $D/pmc_${W}_fetch > $D/${W}_pmc.txt && cat $D/${W}_pmc.txt
