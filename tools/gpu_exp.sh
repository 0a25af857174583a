#!/bin/bash
# partition kernel A timing under PH_DEBUG_FLAGS (results invalid when flags != 0) x tile words x LDS slots
run() {
  echo "flags=$1 tw=$2 slots=$3"
  PH_DEBUG_FLAGS=$1 PH_TILE_WORDS=$2 PH_PART_SLOTS=$3 PH_DEBUG_STAMPS=1 PH_PART_SERIAL=1 timeout -k 10 300 python3 bench.py --workload config3 --steps 2 --warmup 1 --no-cpu 2>&1 | grep -E "stamps" | tail -1 || exit 1
  PH_DEBUG_FLAGS=$1 PH_TILE_WORDS=$2 PH_PART_SLOTS=$3 PH_PART_SERIAL=1 timeout -k 10 300 python3 bench.py --workload config3 --steps 3 --warmup 1 --no-cpu 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('kernel_ms', d['roofline']['kernel_ms'], 'ms_per_step', d['ms_per_step'])" || exit 1
}
for cfg in ${CFGS:-"0 8 8192" "6 8 8192" "2 8 8192" "6 16 8192" "6 32 8192" "6 8 2048"}; do run $cfg; done
