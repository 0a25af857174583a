#!/bin/bash
# partition kernel A timing under the PH_DEBUG_FLAGS experiments (results invalid when flags != 0)
for br in 33554432 2000000000; do
for f in ${FLAGS:-0 6}; do
  echo "batch_rows=$br flags=$f"
  PH_PART_BATCH_ROWS=$br PH_DEBUG_FLAGS=$f PH_DEBUG_STAMPS=1 PH_PART_SERIAL=1 timeout -k 10 300 python3 bench.py --workload config3 --steps 2 --warmup 1 --no-cpu 2>&1 | grep -E "stamps" | tail -1
  PH_PART_BATCH_ROWS=$br PH_DEBUG_FLAGS=$f PH_PART_SERIAL=1 timeout -k 10 300 python3 bench.py --workload config3 --steps 3 --warmup 1 --no-cpu 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('kernel_ms', d['roofline']['kernel_ms'], 'ms_per_step', d['ms_per_step'])"
done
done
