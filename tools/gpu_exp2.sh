#!/bin/bash
# kernel A/B breakdown of the headline query: flags (2 = no flush, 4 = no append; results invalid when != 0)
# x tile words x LDS slots; one line per configuration
set -o pipefail
for cfg in ${CFGS:-0:8:8192 6:8:8192 4:8:8192 2:8:8192 0:16:8192 6:16:8192}; do
  IFS=: read f tw sl wg klo <<< "$cfg"
  r=$(PH_PART_KLO=${klo:-12} PH_PART_WG_PER_CU=${wg:-6} PH_DEBUG_FLAGS=$f PH_TILE_WORDS=$tw PH_PART_SLOTS=$sl PH_PART_SERIAL=1 timeout -k 10 200 python3 bench.py --workload config3 --steps 3 --warmup 1 --no-cpu --no-parity 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('kernel_ms', round(d['roofline']['kernel_ms'],3), 'ms_per_step', round(d['ms_per_step'],3))") || exit 1
  echo "flags=$f tw=$tw slots=$sl wg=${wg:-6} klo=${klo:-12} $r" | tee -a gpurun_out/exp2.txt
done
