#!/bin/bash
# r6: config-3 host-side phases of the step (PH_HOST_TIMES) and a second bench line on a fresh box
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
PH_HOST_TIMES=1 timeout -k 10 300 python -u bench.py --workload config3 --steps 5 --warmup 2 --no-cpu \
  > gpurun_out/r6h_bench.json 2> gpurun_out/r6h_bench.err
rc=$?; echo "rc=$rc"; cat gpurun_out/r6h_bench.json; grep "ph host" gpurun_out/r6h_bench.err | tail -24
exit $rc
