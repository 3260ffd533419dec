#!/bin/bash
# ScanNet stand-in (8 shared-focal pairs in flight) under the latency-oriented
# switches (early continuation, MD lanes per sample, one-sample-per-wave QR), then the
# single-pair cal / sf lines with early continuation on / off.  usage: scannet_ab.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/scab}
mkdir -p "$out"
run() { # name workload env...
  local name=$1 wl=$2; shift 2
  if [ "$wl" = scannet ]; then args="--steps 3 --warmup 1 --no-point-only"; else args="--steps 40 --in-flight 1"; fi
  env "$@" timeout -k 10 200 python bench.py --workload $wl --cpu-budget 0 $args > "$out/$name.json" 2>/dev/null || exit $?
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["value"],1), round(d["ms_per_step"],3))' "$out/$name.json" "$name" || exit 1
}
for r in 1 2; do
  run sc_default$r scannet MADPOSE_NOTHING=1
  run sc_early_forced$r scannet MADPOSE_EARLY_CONT=1x
  run cal_default$r cal MADPOSE_NOTHING=1
  run cal_early0_$r cal MADPOSE_EARLY_CONT=0
  run sf_default$r sf MADPOSE_NOTHING=1
  run sf_early0_$r sf MADPOSE_EARLY_CONT=0
done
