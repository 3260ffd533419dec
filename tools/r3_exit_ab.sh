tools/gpu_steps.sh \
 "400:pytest_gpu:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "200:bench_cal_exit:python bench.py --cpu-budget 0" \
 "200:bench_cal_noexit:MADPOSE_SCORE_EXIT=0 python bench.py --cpu-budget 0" \
 "200:bench_sf_exit:python bench.py --workload sf --cpu-budget 0" \
 "200:bench_sf_noexit:MADPOSE_SCORE_EXIT=0 python bench.py --workload sf --cpu-budget 0" \
 "200:bench_tf_exit:python bench.py --workload tf --cpu-budget 0" \
 "200:bench_tf_noexit:MADPOSE_SCORE_EXIT=0 python bench.py --workload tf --cpu-budget 0"
