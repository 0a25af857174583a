#!/bin/bash
for w in ${WORKLOADS:-config3 config2}; do
  PH_DEBUG_STAMPS=1 PH_PART_SERIAL=1 timeout -k 10 300 python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu 2>&1 | grep -E "stamps|metric" | tail -3 | cut -c1-200
done
