#!/bin/bash
# Round-3 evidence, part 4: the SSB flight with inverted dimension indexes (per-query times + the bench line), then
# rocprofv3 kernel-trace summaries of every workload.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/flight_times.py 60 4 > gpurun_out/r3_flight_inv.txt 2>&1
rc=$?; tail -13 gpurun_out/r3_flight_inv.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload config4 --steps 10 --warmup 3 > gpurun_out/bench_config4.json \
  2> gpurun_out/bench_config4.err
rc=$?; echo "bench config4 rc=$rc"; cut -c1-300 gpurun_out/bench_config4.json; [ $rc -eq 0 ] || exit $rc
for w in ${PROF:-config3 config3-lds config2 config3-agg config4 config5}; do bash tools/gpu_prof.sh $w _r3 || exit $?; done
