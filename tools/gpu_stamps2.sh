#!/bin/bash
# per-workgroup cycle split (stage / decode / sync+flush) of partition kernel A under tuning knobs
for cfg in ${CFGS:-0:8:8192:4}; do
  IFS=: read f tw sl wg <<< "$cfg"
  echo "flags=$f tw=$tw slots=$sl wg=$wg" >> gpurun_out/stamps2.txt
  PH_PART_WG_PER_CU=$wg PH_DEBUG_FLAGS=$f PH_TILE_WORDS=$tw PH_PART_SLOTS=$sl PH_DEBUG_STAMPS=1 PH_PART_SERIAL=1 timeout -k 10 200 python3 bench.py --workload config3 --steps 2 --warmup 1 --no-cpu --no-parity 2>&1 | grep stamps | tail -1 >> gpurun_out/stamps2.txt || exit 1
done
