for cfg in "A:" "S0:MADPOSE_LO_SPECULATE=0" "P1:MADPOSE_SWEEP_PRIORITY=1" "A2:" "S02:MADPOSE_LO_SPECULATE=0" "P12:MADPOSE_SWEEP_PRIORITY=1"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs MADPOSE_LO_TIMING=1 timeout -k 10 200 python bench.py --cpu-budget 0 --in-flight 1 > gpurun_out/lox_$name.json 2> gpurun_out/lox_$name.err || exit 1
done
