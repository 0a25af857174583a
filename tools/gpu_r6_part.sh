#!/bin/bash
# r6: partition-path parity (the fixed-count flush) then a kernel-time A/B of config 3 (fixed flush vs the r5 flush).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "partition" > gpurun_out/r6c_part.log 2>&1
rc=$?
echo "partition tests rc=$rc"; tail -3 gpurun_out/r6c_part.log
[ $rc -eq 0 ] || exit $rc
NO_SQ=1 timeout -k 10 400 bash tools/gpu_kprof.sh "-" "PH_PART_FIXED0=1" "-"
