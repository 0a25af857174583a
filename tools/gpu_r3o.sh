#!/bin/bash
# r3: lean widths (k_agg_reg opt-in) + config3 with rank-atomic batches of 4 (default .so) vs 8 (variant .so),
# config3-lds at L = 16
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lean_widths.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_o.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_o.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/pytest_o.log | head -30; exit $rc; fi
timeout -k 10 300 python3 -u tools/sweep_inproc.py config3 "-" "-" > gpurun_out/r3_sweep_ab4.txt 2>&1
rc=$?; tail -2 gpurun_out/r3_sweep_ab4.txt; [ $rc -eq 0 ] || exit $rc
PH_LIB_PATH=$(pwd)/pinot_amd/libpinot_hip_ab8.so timeout -k 10 300 python3 -u tools/sweep_inproc.py config3 "-" "-" \
  > gpurun_out/r3_sweep_ab8.txt 2>&1
rc=$?; tail -2 gpurun_out/r3_sweep_ab8.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/sweep_inproc.py config3-lds "-" "PH_GROUP_REG_LG=5" "-" > gpurun_out/r3_sweep_lds.txt 2>&1
rc=$?; tail -3 gpurun_out/r3_sweep_lds.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/flight_times.py 60 4 > gpurun_out/r3_flight.txt 2>&1
rc=$?; tail -13 gpurun_out/r3_flight.txt; exit $rc
