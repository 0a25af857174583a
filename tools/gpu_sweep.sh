#!/bin/bash
# kernel time of the headline query under tuning knobs (serial A/B, single batch by default)
for tw in ${TWS:-8 16}; do for sl in ${SLOTS:-4096 8192}; do
  r=$(PH_TILE_WORDS=$tw PH_PART_SLOTS=$sl PH_PART_BATCH_ROWS=${BR:-2000000000} PH_PART_SERIAL=1 timeout -k 10 300 python3 bench.py --workload config3 --steps 3 --warmup 1 --no-cpu 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('%.3f %.3f' % (d[\"roofline\"][\"kernel_ms\"], d[\"ms_per_step\"]))")
  echo "tw=$tw slots=$sl kernel_ms/ms_per_step=$r"
done; done
