#!/bin/bash
# Config-3 sweep: each CFGS item "FLAGS:TILE_WORDS:RING_LOG2:WG_PER_CU:KLO" is one bench run with kernels A and
# B serialised (PH_PART_SERIAL=1); debug flags (results invalid when != 0): 2 no flush, 4 no append,
# 8 no rank atomic, 16 no key/value decode.  One line per configuration in gpurun_out/sweep.txt.
set -o pipefail
mkdir -p gpurun_out
for cfg in ${CFGS:-0:16:5:6:12}; do
  IFS=: read f tw rl wg klo <<< "$cfg"
  r=$(PH_PART_KLO=${klo:-12} PH_PART_WG_PER_CU=${wg:-6} PH_DEBUG_FLAGS=$f PH_TILE_WORDS=$tw PH_PART_RING_LOG2=${rl:-5} \
      PH_PART_SERIAL=1 timeout -k 10 200 python3 bench.py --workload ${W:-config3} --steps 3 --warmup 1 --no-cpu \
      --no-parity 2>gpurun_out/sweep.err | python3 -c "import json,sys; d=json.load(sys.stdin); print('kernel_ms', round(d['roofline']['kernel_ms'],3), 'ms_per_step', round(d['ms_per_step'],3))") || { tail -5 gpurun_out/sweep.err; exit 1; }
  echo "flags=$f tw=$tw ring=$rl wg=${wg:-6} klo=${klo:-12} $r" | tee -a gpurun_out/sweep.txt
done
