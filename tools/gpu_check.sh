#!/bin/bash
# GPU-box round: parity suite, then one bench line per workload.  Stops at the first crash / timeout.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=30 --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
for w in ${WORKLOADS:-config2 config3-agg config3-lds config3}; do
  timeout -k 10 400 python -u bench.py --workload $w --steps ${STEPS:-5} --warmup 2 --cpu-seconds ${CPU_SECS:-5} \
    > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err
  rc=$?
  echo "bench $w rc=$rc"
  cat gpurun_out/bench_$w.json
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_$w.err; exit $rc; fi
done
