#!/bin/bash
# r3: k_agg_reg restructured (unpack + one register set), kernel B per-lane dummy keys; parity first
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lean_widths.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_n.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_n.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/pytest_n.log | head -30; exit $rc; fi
timeout -k 10 300 python3 -u tools/sweep_inproc.py config3-agg "-" "PH_AGG_LDS=1" "-" > gpurun_out/r3_sweep_agg.txt 2>&1
rc=$?; tail -3 gpurun_out/r3_sweep_agg.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/sweep_inproc.py config3 "-" "PH_PART_MM_BLIND=1" "-" > gpurun_out/r3_sweep_b.txt 2>&1
rc=$?; tail -3 gpurun_out/r3_sweep_b.txt; exit $rc
