# Round-6 final measurement set (repo root on the box): PMC fit of score_batch, the four
# bench lines (CPU legs included), rocprofv3 kernel statistics of cal / sf / tf, per-kernel
# PMC of the shared-focal chain.  usage: bash tools/gpu_final.sh <dir under gpurun_out>
set -o pipefail
cd $GRAFT_REPO_ROOT
N=$1; D=gpurun_out/$N; mkdir -p $D
bash tools/pmc_passes.sh $D/pmc || exit $?
SQ=$(find $D/pmc -name 'sq_counter_collection.csv' | head -1); FE=$(find $D/pmc -name 'fetch_counter_collection.csv' | head -1)
python3 tools/pmc_score.py "$SQ" "$FE" $D/pmc_score_batch.json "profiles/r06/$N/pmc (tools/pmc_passes.sh on the round-6 final tree)" || exit $?
mkdir -p profiles/r06/$N && cp $D/pmc_score_batch.json profiles/r06/pmc_score_batch.json || exit $?
bash tools/gpu_r6_bench.sh $N || exit $?
bash tools/gpu_prof.sh $N cal --steps 20 || exit $?
bash tools/gpu_prof.sh $N sf --steps 10 || exit $?
bash tools/gpu_prof.sh $N tf --steps 10 || exit $?
bash tools/pmc_kernels.sh $N sf || exit $?
