# Repeated short bench lines (no CPU legs) for A/B comparisons across builds:
# usage: tools/bench_rep.sh <workload> <repeats>
wl=${1:-cal}; n=${2:-3}
for i in $(seq "$n"); do
  timeout -k 10 120 python bench.py --workload "$wl" --cpu-budget 0 --in-flight 1 --steps 80 > gpurun_out/rep_${wl}_${i}.json 2>/dev/null || exit $?
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["value"]), round(d["ms_per_step"],3), {k: round(v,3) for k,v in d["ms_per_pair"].items()})' gpurun_out/rep_${wl}_${i}.json "$wl" || exit 1
done
MADPOSE_LO_TIMING=1 timeout -k 10 120 python bench.py --workload "$wl" --cpu-budget 0 --in-flight 1 --steps 20 2>&1 >/dev/null | grep 'LO:' | tail -3 || true
