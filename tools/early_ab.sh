#!/bin/bash
# early continuation: GPU suite, then A/B against MADPOSE_EARLY_CONT=0 on cal / sf / tf
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/early_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/early_pytest.log; [ $rc -eq 0 ] || exit $rc
tools/cal_ab.sh early "on1:-" "off1:MADPOSE_EARLY_CONT=0" "on2:-" "off2:MADPOSE_EARLY_CONT=0" "on3:-" "off3:MADPOSE_EARLY_CONT=0" || exit 1
WL=sf STEPS=40 tools/cal_ab.sh early_sf "on1:-" "off1:MADPOSE_EARLY_CONT=0" "on2:-" "off2:MADPOSE_EARLY_CONT=0" || exit 1
WL=tf STEPS=40 tools/cal_ab.sh early_tf "on1:-" "off1:MADPOSE_EARLY_CONT=0" "on2:-" "off2:MADPOSE_EARLY_CONT=0" || exit 1
MADPOSE_LO_TIMING=1 timeout -k 10 120 python bench.py --cpu-budget 0 --in-flight 1 --steps 10 2> gpurun_out/early_timing_cal.log > /dev/null; grep "pair:" gpurun_out/early_timing_cal.log | tail -4
