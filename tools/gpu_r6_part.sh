#!/bin/bash
# r6: partition-path parity (kernel A ring sets, kernel B pipelined loads, options instead of env in the library)
# then a kernel-time A/B of config 3.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_lean_widths.py -k "partition or lean" > gpurun_out/r6d_part.log 2>&1
rc=$?
echo "partition + lean tests rc=$rc"; tail -3 gpurun_out/r6d_part.log
[ $rc -eq 0 ] || exit $rc
NO_SQ=1 timeout -k 10 400 bash tools/gpu_kprof.sh "-" "PH_PART_SETS=1" "PH_PART_SETS=2"
