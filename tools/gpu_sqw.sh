#!/bin/bash
# SQ counters (two passes) of one bench workload, any kind (flights included): per-kernel sums (tools/sq_summary.py).
W=${1:-config4-scan}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/sqw_$W
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- \
    python3 $ROOT/bench.py --workload $W --steps 1 --warmup 0 --no-cpu --no-parity > $OUT/p$i.json 2> $OUT/p$i.err
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.err; exit $rc; fi
done
python3 $ROOT/tools/sq_summary.py $OUT
