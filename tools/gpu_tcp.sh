#!/bin/bash
# TLB / L1 / latency counters of the scan kernels for one bench workload: TCP_* passes (<= 4 TCP counters each),
# each under its own time limit; per-kernel sums printed by tools/sq_summary.py.
W=${1:-config3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/tcp_$W
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
P1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
P2="TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- \
    python3 $ROOT/bench.py --workload $W --steps 1 --warmup 0 --no-cpu --no-parity > $OUT/p$i.json 2> $OUT/p$i.err
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.err; exit $rc; fi
done
python3 $ROOT/tools/sq_summary.py $OUT
