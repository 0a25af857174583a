#!/bin/bash
# Round evidence (TAG, default r6f), in phases that each fit one gpurun call (PHASE = tests | bench | prof | pmc):
#   tests: the full -m gpu suite + smoke();  bench: one bench line per workload (BENCH list);
#   prof:  rocprofv3 kernel-trace summaries (PROF list);  pmc: FETCH_SIZE / WRITE_SIZE passes (PMC list).
# Everything lands under gpurun_out/${TAG}_* ; every GPU step has its own time limit and the script stops at the first
# failing step.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
TAG=${TAG:-r6f}
case ${PHASE:-tests} in
  tests)
    timeout -k 10 720 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/${TAG}_pytest_gpu.log 2>&1
    rc=$?; tail -5 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/${TAG}_smoke.log; exit $rc ;;
  bench)
    for w in ${BENCH:-config3 config2 config3-agg config3-lds config1}; do
      timeout -k 10 ${BTIME:-400} python -u bench.py --workload $w --steps ${STEPS:-10} --warmup 3 --cpu-seconds ${CPU_SECS:-10} \
        > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err
      rc=$?; echo "bench $w rc=$rc"; cat gpurun_out/${TAG}_bench_$w.json
      [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench_$w.err; exit $rc; }
    done ;;
  prof)
    for w in ${PROF:-config3 config2}; do bash tools/gpu_prof.sh $w _${TAG} || exit $?; done ;;
  pmc)
    # (each summary is also copied into this box's profiles/ so a bench phase later in the same call reports it)
    for w in ${PMC:-config3}; do bash tools/gpu_pmc.sh $w || exit $?; cat gpurun_out/pmc_$w.json;
      cp gpurun_out/pmc_$w.json profiles/${TAG%f}_pmc_$w.json; done ;;
  multi)
    timeout -k 10 400 python -u bench.py --workload config3 --devices 0,0 --steps 5 --warmup 2 --no-cpu \
      > gpurun_out/${TAG}_bench_config3_devices00.json 2> gpurun_out/${TAG}_bench_config3_devices00.err
    rc=$?; echo "bench devices 0,0 rc=$rc"; cat gpurun_out/${TAG}_bench_config3_devices00.json; exit $rc ;;
esac
