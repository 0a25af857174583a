#!/bin/bash
# r3: k_group_reg branch-free atomics -- lean-width parity + GPU parity, then config3-lds vs k_group_lds_lean
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lean_widths.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_l.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_l.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/pytest_l.log | head -30; exit $rc; fi
timeout -k 10 300 python3 -u tools/sweep_inproc.py config3-lds "-" "PH_LDS_LEAN=1" "-" \
  > gpurun_out/r3_sweep_lds.txt 2>&1
rc=$?; tail -4 gpurun_out/r3_sweep_lds.txt; exit $rc
