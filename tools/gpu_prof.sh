#!/bin/bash
# rocprofv3 kernel-trace summary of one bench workload (no PMC counters in this pass).
W=${1:-config3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$W
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 $ROOT/bench.py --workload $W --steps 3 --warmup 1 --no-cpu > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "rocprof $W rc=$rc"
cat $OUT/bench.json
find $OUT -name "*kernel_stats.csv" | head -3 | while read f; do echo "== $f"; head -20 "$f"; done
exit $rc
