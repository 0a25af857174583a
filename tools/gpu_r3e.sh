#!/bin/bash
# r3: k_part_reg breakdown -- kernel trace of config3, then the knob sweep
mkdir -p gpurun_out
bash tools/gpu_prof.sh config3 _reg || exit $?
timeout -k 10 400 python3 -u tools/sweep_inproc.py config3 "-" "PH_PART_ROUNDS=1,PH_PART_RING_LOG2=6" \
  "PH_PART_WG_PER_CU=1" "PH_PART_LDS=1" "-" > gpurun_out/r3_sweep_reg.txt 2>&1
rc=$?; tail -8 gpurun_out/r3_sweep_reg.txt; exit $rc
