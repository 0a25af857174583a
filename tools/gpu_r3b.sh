#!/bin/bash
# r3: kernel A two-deep pipeline -- parity of the partition tests under PH_PART_DEPTH=2, then the config-3 sweep
mkdir -p gpurun_out
PH_PART_DEPTH=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q \
  -k "partition or config3 or limit" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_depth2.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_depth2.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/pytest_depth2.log | head -30; exit $rc; fi
timeout -k 10 500 python3 -u tools/sweep_inproc.py config3 "-" "PH_PART_DEPTH=2" "PH_PART_DEPTH=2,PH_PART_DBG=2" \
  "PH_PART_DEPTH=2,PH_TILE_WORDS=8" "PH_PART_DEPTH=2,PH_TILE_WORDS=16" "-" "PH_PART_DEPTH=2" \
  "PH_PART_DEPTH=2,PH_PART_SERIAL=1" > gpurun_out/r3_sweep1.txt 2>&1
rc=$?; tail -9 gpurun_out/r3_sweep1.txt; exit $rc
