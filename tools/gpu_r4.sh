#!/bin/bash
# Round-4 iteration recipe: selected -m gpu tests (TESTS = pytest -k expression, FILES = test files), then an
# in-process knob sweep of a bench workload (SWEEP = "workload setting ..."; settings as tools/sweep_inproc.py).
# Output under gpurun_out/r4_<TAG>.*; stops at the first failing step.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
TAG=${TAG:-it}
if [ -n "$FILES" ]; then
  timeout -k 10 ${TTIME:-600} python -u -m pytest $FILES -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider ${TESTS:+-k "$TESTS"} > gpurun_out/r4_$TAG.pytest.log 2>&1
  rc=$?; tail -5 gpurun_out/r4_$TAG.pytest.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$SWEEP" ]; then
  timeout -k 10 ${STIME:-400} python3 -u tools/sweep_inproc.py $SWEEP > gpurun_out/r4_$TAG.sweep.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/r4_$TAG.sweep.txt; [ $rc -eq 0 ] || exit $rc
fi
exit 0
