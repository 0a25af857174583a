#!/bin/bash
# HBM traffic of one bench workload from rocprofv3 PMC counters (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and
# WRITE_SIZE in separate passes (each with its own time limit), then tools/pmc_summary.py writes
# gpurun_out/pmc_<workload>.json (copy to profiles/ to have bench.py report it as roofline.traffic).
W=${1:-config3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$W
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $OUT/$C -o run -- \
    python3 $ROOT/bench.py --workload $W --steps 1 --warmup 1 --no-cpu > $OUT/$C.json 2> $OUT/$C.err
  rc=$?
  echo "pmc $C rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$C.err; exit $rc; fi
done
python3 $ROOT/tools/pmc_summary.py $W $OUT $ROOT/gpurun_out/pmc_$W.json
