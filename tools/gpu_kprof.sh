#!/bin/bash
# Kernel times + SQ counters of one workload in one process (tools/sweep_inproc.py, settings as arguments):
# a kernel-trace pass, then the two SQ passes of tools/gpu_sq.sh's counter sets, each under its own time limit.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
W=${W:-config3}
OUT=$ROOT/gpurun_out/kprof_$W
mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 $ROOT/tools/sweep_inproc.py $W "$@" > $OUT/kt.txt 2>&1 || { tail -5 $OUT/kt.txt; exit 1; }
cat $OUT/kt.txt | grep device_ms
python3 - $OUT/kt <<'EOF'
import csv, glob, sys
f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True))
for r in csv.DictReader(open(f[-1])):
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>5s} avg_ms {float(r['AverageNs'])/1e6:8.3f} tot_ms {float(r['TotalDurationNs'])/1e6:9.2f}")
EOF
[ -n "$NO_SQ" ] && exit 0
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  SWEEP_ITERS=1 timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- \
    python3 $ROOT/tools/sweep_inproc.py $W "$@" > $OUT/p$i.txt 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.txt; exit $rc; fi
done
python3 $ROOT/tools/sq_summary.py $OUT
