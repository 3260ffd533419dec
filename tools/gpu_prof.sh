# rocprofv3 kernel statistics of one bench workload: gpurun_out/$1/$2_kernel_stats.csv
# usage (repo root on the box): bash tools/gpu_prof.sh <dir> <workload> [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/$1; W=$2; shift 2
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof_$W -o $W -- python3 $R/bench.py --workload $W --cpu-budget 0 --in-flight 1 "$@" > $D/prof_$W.log 2>&1 || exit $?
cd $R && python3 tools/prof_summary.py $D/prof_$W $D/${W}_kernel_stats.csv > $D/${W}_summary.log && head -14 $D/${W}_summary.log
