#!/bin/bash
# r6: config-3 step variance -- two default-length bench runs with the library's phase stamps
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for i in 1 2; do
  PH_HOST_TIMES=1 timeout -k 10 300 python -u bench.py --workload config3 --steps 20 --warmup 3 --no-cpu --no-parity \
    > gpurun_out/r6v_$i.json 2> gpurun_out/r6v_$i.err
  rc=$?; echo "run $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 -c "
import json
d=json.loads(open('gpurun_out/r6v_$i.json').readline()); print(round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))"
  grep "ph host" gpurun_out/r6v_$i.err | tail -6
done
numactl -H 2>/dev/null | head -4; cat /sys/class/drm/card*/device/numa_node 2>/dev/null | head -3
exit 0
