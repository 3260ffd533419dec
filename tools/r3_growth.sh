tools/gpu_steps.sh \
 "60:eig_8192:tools/eig6_bench 8192" \
 "60:eig_2048:tools/eig6_bench 2048" \
 "60:eig_64:tools/eig6_bench 64" \
 "150:cal_g4:python bench.py --cpu-budget 0 --in-flight 1" \
 "150:cal_g1:MADPOSE_BATCH_GROWTH=1 python bench.py --cpu-budget 0 --in-flight 1" \
 "150:cal_g05:MADPOSE_BATCH_GROWTH=0.5 python bench.py --cpu-budget 0 --in-flight 1" \
 "150:sf_g4:python bench.py --workload sf --cpu-budget 0 --in-flight 1" \
 "150:sf_g1:MADPOSE_BATCH_GROWTH=1 python bench.py --workload sf --cpu-budget 0 --in-flight 1" \
 "150:tf_g4:python bench.py --workload tf --cpu-budget 0 --in-flight 1" \
 "150:tf_g1:MADPOSE_BATCH_GROWTH=1 python bench.py --workload tf --cpu-budget 0 --in-flight 1"
