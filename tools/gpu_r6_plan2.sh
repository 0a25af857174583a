#!/bin/bash
# r6: host phases (PH_HOST_TIMES) of the aggregation-only and small workloads
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for w in config2 config3-agg config3-lds config1; do
  PH_HOST_TIMES=1 timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 3 --no-cpu --no-parity \
    > gpurun_out/r6p2_$w.json 2> gpurun_out/r6p2_$w.err
  rc=$?; echo "$w rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 -c "
import json; d=json.loads(open('gpurun_out/r6p2_$w.json').readline()); print('ms/step', round(d['ms_per_step'],3), 'kernel', round(d['roofline']['kernel_ms'],3))"
  grep "ph host" gpurun_out/r6p2_$w.err | tail -18
done
exit 0
