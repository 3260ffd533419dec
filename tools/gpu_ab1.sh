set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/ab14; mkdir -p $D
bash tools/env_ab.sh $D sf 3 base=MADPOSE_LIB_VARIANT=base qr=MADPOSE_NOTHING=1 r4=MADPOSE_LIB_VARIANT=r4 || exit $?
for rep in 1 2; do for v in base qr r4; do
  e=MADPOSE_NOTHING=1; [ $v = base ] && e=MADPOSE_LIB_VARIANT=base; [ $v = r4 ] && e=MADPOSE_LIB_VARIANT=r4
  env $e timeout -k 10 300 python bench.py --workload scannet --cpu-budget 0 --steps 3 --warmup 1 --no-point-only > $D/sn_${v}_$rep.json 2>/dev/null || exit $?
  python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d["value"],1), round(d["ms_per_step"],3))' $D/sn_${v}_$rep.json "sn $v" || exit 1
done; done
