#!/bin/bash
# Round-3 evidence, part 1: the full -m gpu suite, smoke, PMC traffic (FETCH_SIZE / WRITE_SIZE passes) of the
# headline and the LDS group-by.  Stops at the first failure.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 150 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
for w in ${PMC:-config3 config3-lds}; do bash tools/gpu_pmc.sh $w || exit $?; done
