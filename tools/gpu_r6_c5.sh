#!/bin/bash
# r6: config-5 step phases (PH_HOST_TIMES), twice
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for i in 1 2; do
  PH_HOST_TIMES=1 timeout -k 10 400 python -u bench.py --workload config5 --steps 10 --warmup 3 --no-cpu --no-parity \
    > gpurun_out/r6c5_$i.json 2> gpurun_out/r6c5_$i.err
  rc=$?; echo "run $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 -c "
import json
d=json.loads(open('gpurun_out/r6c5_$i.json').readline()); print(round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))"
  grep "ph host" gpurun_out/r6c5_$i.err | tail -7
done
exit 0
