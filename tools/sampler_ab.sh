for i in 1 2 3; do
 for v in 1 0; do
  echo "cal two_pass=$v: $(MADPOSE_SAMPLER_TWO_PASS=$v timeout -k 10 120 python bench.py --cpu-budget 0 --in-flight 1 --steps 80 | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["value"]), round(d["ms_per_step"],3), d["ms_per_pair"])')" || exit 1
 done
done
for v in 1 0; do
  echo "sf two_pass=$v: $(MADPOSE_SAMPLER_TWO_PASS=$v timeout -k 10 120 python bench.py --workload sf --cpu-budget 0 --in-flight 1 | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d["value"]), round(d["ms_per_step"],3), d["ms_per_pair"])')" || exit 1
done
