#!/bin/bash
# r6: partition-path parity (kernel A ring sets, kernel B pipelined loads) then a kernel-time A/B of config 3.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "partition" > gpurun_out/r6d_part.log 2>&1
rc=$?
echo "partition tests rc=$rc"; tail -3 gpurun_out/r6d_part.log
[ $rc -eq 0 ] || exit $rc
PH_PART_SETS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "partition" > gpurun_out/r6d_part1.log 2>&1
rc=$?
echo "partition tests (one ring set) rc=$rc"; tail -2 gpurun_out/r6d_part1.log
[ $rc -eq 0 ] || exit $rc
NO_SQ=1 timeout -k 10 400 bash tools/gpu_kprof.sh "-" "PH_PART_SETS=1" "PH_PART_SETS=2"
