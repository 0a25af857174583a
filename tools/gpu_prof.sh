#!/bin/bash
# rocprofv3 kernel-trace summary of one bench workload (no PMC counters in this pass).
W=${1:-config3}
TAG=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$W$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 $ROOT/bench.py --workload $W --steps 3 --warmup 1 --no-cpu > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "rocprof $W$TAG rc=$rc"
python3 -c "import json,sys; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print('ms/step %.3f kernel_ms %.3f frac %.3f GB/s %.0f' % (d['ms_per_step'], r['kernel_ms'], r['frac'], r['achieved']))" || tail -5 $OUT/bench.err
python3 - $OUT <<'PY'
import csv, glob, sys
f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True))
for r in list(csv.DictReader(open(f[-1])))[:14]:
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>5s} avg_ms {float(r['AverageNs'])/1e6:8.3f} tot_ms {float(r['TotalDurationNs'])/1e6:9.2f}")
PY
exit $rc
