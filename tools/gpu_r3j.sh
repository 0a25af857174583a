#!/bin/bash
# r3: new-feature GPU tests (range index, segment trim, k_count_reg widths, applyAnd statistic), then the config2
# count-kernel comparison and the config3 append-variant sweep
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_range_index.py tests/test_gpu_trim.py tests/test_gpu_lean_widths.py \
  tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_raw.py tests/test_gpu_loader.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_j.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_j.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/pytest_j.log | head -30; exit $rc; fi
timeout -k 10 300 python3 -u tools/sweep_inproc.py config2 "-" "PH_COUNT_GENERIC=1" "-" "PH_COUNT_GENERIC=1" \
  > gpurun_out/r3_sweep_count.txt 2>&1
rc=$?; tail -5 gpurun_out/r3_sweep_count.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u tools/sweep_inproc.py config3 "-" "PH_PART_VARIANT=1" "PH_PART_VARIANT=2" "PH_PART_VARIANT=3" \
  "PH_PART_KLO=13,PH_PART_ROUNDS=1,PH_PART_RING_LOG2=6" "PH_PART_KLO=13,PH_PART_ROUNDS=1,PH_PART_RING_LOG2=6,PH_PART_SLICES=2" \
  "PH_PART_SLICES=2" "-" > gpurun_out/r3_sweep_var.txt 2>&1
rc=$?; tail -9 gpurun_out/r3_sweep_var.txt; exit $rc
