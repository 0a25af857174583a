#!/bin/bash
# Round-3 evidence, part 2: config / lean-width parity at HEAD, config-2 PMC (register-direct calibration), then one
# bench line per workload and the SSB flight's per-query times.  Stops at the first failure.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_lean_widths.py -m gpu -q --maxfail=5 \
  --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ev2.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_ev2.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc.sh config2 || exit $?
for w in ${WORKLOADS:-config3 config2 config3-agg config3-lds config1 config4 config5}; do
  timeout -k 10 400 python -u bench.py --workload $w --steps ${STEPS:-10} --warmup 3 \
    > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err
  rc=$?
  echo "bench $w rc=$rc"; cat gpurun_out/bench_$w.json | cut -c1-400
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_$w.err; exit $rc; fi
done
timeout -k 10 300 python3 -u tools/flight_times.py 60 4 > gpurun_out/r3_flight.txt 2>&1
rc=$?; tail -13 gpurun_out/r3_flight.txt; exit $rc
