#!/bin/bash
# r6: kernel-trace summary of the scan-dimension flight (tools/ssb_host_times.py) under rocprofv3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out/r6_dfaprof${W:-}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r6_dfaprof${W:-} -o run -- \
  python3 $ROOT/tools/ssb_host_times.py ${W:-config4-scan} > $ROOT/gpurun_out/r6_dfaprof${W:-}/out.txt 2> $ROOT/gpurun_out/r6_dfaprof${W:-}/err.txt
rc=$?; echo "rc=$rc"
f=$(find $ROOT/gpurun_out/r6_dfaprof${W:-} -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -12 "$f" | cut -c1-220
exit $rc
