#!/bin/bash
# r6: scan-dimension SSB flight per query with the sparse kernels' register-direct leaf width forced to 4 and 8 vs the
# planner's choice (2 for <= 8-bit leaves)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for V in default 4 8; do
  if [ $V = default ]; then unset PH_SPARSE_C; else export PH_SPARSE_C=$V; fi
  timeout -k 10 400 python -u tools/ssb_host_times.py config4-scan > gpurun_out/r6c_$V.txt 2> gpurun_out/r6c_$V.err
  rc=$?; echo "sparse_c $V rc=$rc"; [ $rc -ne 0 ] && exit $rc
  cat gpurun_out/r6c_$V.txt
done
exit 0
