#!/bin/bash
# r3 re-entry: full GPU parity suite + smoke + bench lines at HEAD.  Stops at the first crash / timeout.
mkdir -p gpurun_out
WORKLOADS=${WORKLOADS:-"config3 config4 config5"} bash tools/gpu_check.sh || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; exit $rc
