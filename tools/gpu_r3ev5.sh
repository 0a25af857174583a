#!/bin/bash
# Round-3 evidence, part 5 (HEAD): the full -m gpu suite, smoke, the SSB flight (per-query + bench line), the lean
# aggregation vs its LDS / generic forms, config-5 PMC at 4B rows.  Stops at the first failure.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 150 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/flight_times.py 60 4 > gpurun_out/r3_flight_inv.txt 2>&1
rc=$?; tail -13 gpurun_out/r3_flight_inv.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload config4 --steps 10 --warmup 3 > gpurun_out/bench_config4.json \
  2> gpurun_out/bench_config4.err
rc=$?; echo "bench config4 rc=$rc"; cut -c1-300 gpurun_out/bench_config4.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/sweep_inproc.py config3-agg "-" "PH_AGG_GENERIC=1" "-" > gpurun_out/r3_sweep_agg.txt 2>&1
rc=$?; tail -3 gpurun_out/r3_sweep_agg.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc.sh config5
