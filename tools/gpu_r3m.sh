#!/bin/bash
# r3: kernel B batched min/max reads (+ blind knob), k_group_reg timing knobs; parity first
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lean_widths.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_m.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_m.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/pytest_m.log | head -30; exit $rc; fi
timeout -k 10 300 python3 -u tools/sweep_inproc.py config3 "-" "PH_PART_MM_BLIND=1" "PH_PART_SERIAL=1" "-" \
  > gpurun_out/r3_sweep_b.txt 2>&1
rc=$?; tail -4 gpurun_out/r3_sweep_b.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/sweep_inproc.py config3-lds "-" "PH_GROUP_REG_DBG=1" "PH_GROUP_REG_LG=4" \
  "PH_GROUP_REG_LG=3" "PH_LDS_LEAN=1" "-" > gpurun_out/r3_sweep_lds.txt 2>&1
rc=$?; tail -6 gpurun_out/r3_sweep_lds.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/sweep_inproc.py config3-agg "-" "PH_AGG_LDS=1" "-" > gpurun_out/r3_sweep_agg.txt 2>&1
rc=$?; tail -3 gpurun_out/r3_sweep_agg.txt; exit $rc
