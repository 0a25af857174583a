#!/bin/bash
# r3: k_part_reg component timing (PH_PART_DBG: 2 no appends, 8 no append rounds) at 166 VGPRs (3 waves / SIMD)
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/sweep_inproc.py config3 "-" "PH_PART_DBG=2" "PH_PART_DBG=8" "PH_PART_WG_PER_CU=2" \
  "PH_PART_ROUNDS=1,PH_PART_RING_LOG2=6" "PH_PART_SERIAL=1" "-" > gpurun_out/r3_sweep_reg2.txt 2>&1
rc=$?; tail -8 gpurun_out/r3_sweep_reg2.txt; exit $rc
