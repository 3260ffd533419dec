# LM-pool spin with two bench ranks on one card (gloo rehearsal): ScanNet stand-in
# pairs/s at MADPOSE_LO_SPIN = 300 (default) and 0 (block at once), one line each
for spin in 300 0 300 0; do
  MADPOSE_LO_SPIN=$spin MADPOSE_BENCH_DIST_BACKEND=gloo MADPOSE_BENCH_DEVICE=0 timeout -k 10 240 \
    python bench.py --gpus 2 --workload scannet --cpu-budget 0 --no-point-only --steps 4 --warmup 1 > gpurun_out/spin_$spin.json 2>/dev/null || exit $?
  python -c 'import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); print("spin", sys.argv[2], "n_gpus", d["n_gpus"], "pairs/s", round(d["value"],1), "ms/step", round(d["ms_per_step"],1))' gpurun_out/spin_$spin.json $spin || exit 1
done
