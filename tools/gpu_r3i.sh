#!/bin/bash
# r3: range-index, raw, loader, parity (applyAnd statistic) and config tests, then the k_part_reg append-variant / occupancy / partition-size sweep
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_range_index.py tests/test_gpu_trim.py tests/test_gpu_raw.py tests/test_gpu_loader.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ri.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ri.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/pytest_ri.log | head -30; exit $rc; fi
timeout -k 10 500 python3 -u tools/sweep_inproc.py config3 "-" "PH_PART_VARIANT=1" "PH_PART_VARIANT=2" "PH_PART_VARIANT=3" \
  "PH_PART_KLO=13,PH_PART_ROUNDS=1,PH_PART_RING_LOG2=6" "PH_PART_KLO=13,PH_PART_ROUNDS=1,PH_PART_RING_LOG2=6,PH_PART_SLICES=2" \
  "PH_PART_KLO=13,PH_PART_ROUNDS=1,PH_PART_RING_LOG2=6,PH_PART_VARIANT=1" "PH_PART_SLICES=2" "-" \
  > gpurun_out/r3_sweep_var.txt 2>&1
rc=$?; tail -10 gpurun_out/r3_sweep_var.txt; exit $rc
