#!/bin/bash
# r3 final: the full -m gpu suite and smoke at HEAD
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 150 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; exit $rc
