#!/bin/bash
# r6: kernel-trace summary of the scan-dimension flight (tools/ssb_host_times.py) under rocprofv3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out/r6_dfaprof
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r6_dfaprof -o run -- \
  python3 $ROOT/tools/ssb_host_times.py config4-scan > $ROOT/gpurun_out/r6_dfaprof/out.txt 2> $ROOT/gpurun_out/r6_dfaprof/err.txt
rc=$?; echo "rc=$rc"
f=$(find $ROOT/gpurun_out/r6_dfaprof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -12 "$f" | cut -c1-220
exit $rc
