#!/bin/bash
# Kernel-B slice sweep on config 3: one bench run per PH_PART_SLICES value (A unchanged, B's grid and merge
# change); one line per value in gpurun_out/slices.txt.
set -o pipefail
mkdir -p gpurun_out
for s in ${SLICES:-1 2 3 4 6}; do
  r=$(PH_PART_SLICES=$s timeout -k 10 200 python3 bench.py --workload config3 --steps 5 --warmup 1 --no-cpu \
      --no-parity 2>gpurun_out/slices.err | python3 -c "import json,sys; d=json.load(sys.stdin); print('kernel_ms', round(d['roofline']['kernel_ms'],3), 'ms_per_step', round(d['ms_per_step'],3))") || { tail -5 gpurun_out/slices.err; exit 1; }
  echo "slices=$s $r" | tee -a gpurun_out/slices.txt
done
