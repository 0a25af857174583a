#!/bin/bash
# Partitioned group-by iteration: its parity tests, then per-kernel times (A and B serialised) and the
# WRITE_SIZE / FETCH_SIZE of the headline workload.  Extra env (PH_*) passes through to bench.py.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "${TESTS:-partition or global_table or large_group or smoke}" > gpurun_out/pytest_part.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_part.log; [ $rc -eq 0 ] || exit $rc
PH_PART_SERIAL=1 bash tools/gpu_prof.sh config3 serial || exit $?
if [ -n "$PMC" ]; then bash tools/gpu_pmc.sh config3 || exit $?; cat gpurun_out/pmc_config3.json; fi
