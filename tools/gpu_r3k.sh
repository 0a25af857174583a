#!/bin/bash
# r3: k_group_reg (register-direct LDS group-by) -- lean-width parity, the GPU parity/config suites, then the
# config3-lds comparison against k_group_lds_lean and the SSB flight
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lean_widths.py tests/test_gpu_parity.py tests/test_gpu_configs.py \
  -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_k.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_k.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/pytest_k.log | head -30; exit $rc; fi
timeout -k 10 300 python3 -u tools/sweep_inproc.py config3-lds "-" "PH_LDS_LEAN=1" "-" "PH_LDS_LEAN=1" \
  > gpurun_out/r3_sweep_lds.txt 2>&1
rc=$?; tail -5 gpurun_out/r3_sweep_lds.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/sweep_inproc.py config3 "-" "PH_PART_BATCH_ROWS=100000000" \
  "PH_PART_BATCH_ROWS=100000000,PH_PART_WG_PER_CU=2" "PH_PART_BATCH_ROWS=250000000" "PH_PART_SERIAL=1" "-" \
  > gpurun_out/r3_sweep_batch.txt 2>&1
rc=$?; tail -7 gpurun_out/r3_sweep_batch.txt; exit $rc
