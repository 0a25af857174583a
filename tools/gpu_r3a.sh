#!/bin/bash
# r3: GPU parity suite, then the config-3 knob sweep (baseline breakdown).  Stops at the first failure.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 500 python3 -u tools/sweep_inproc.py config3 "-" "PH_PART_DBG=2" "PH_PART_DBG=1" "PH_PART_SERIAL=1" \
  "PH_PART_DBG=4,PH_PART_SERIAL=1" > gpurun_out/r3_sweep0.txt 2>&1
rc=$?; tail -8 gpurun_out/r3_sweep0.txt; exit $rc
