#!/bin/bash
# Where kernel A's waves spend their cycles (PH_DEBUG_STAMPS, wave 0 of each workgroup): one line per debug-flag
# setting (flags as tools/gpu_sweep.sh; results invalid when != 0).
mkdir -p gpurun_out
for f in ${FLAGS:-0 16 8 6}; do
  echo "flags=$f $(PH_DEBUG_FLAGS=$f PH_DEBUG_STAMPS=1 PH_PART_SERIAL=1 timeout -k 10 200 python3 bench.py --workload ${W:-config3} \
    --steps 2 --warmup 1 --no-cpu --no-parity 2>&1 | grep -E "stamps" | tail -1)" | tee -a gpurun_out/stamps.txt || exit 1
done
