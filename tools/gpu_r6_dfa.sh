#!/bin/bash
# r6: the per-word AND-walk kernel -- its parity tests, then the scan-dimension flight's per-query split
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_and_walk.py \
  tests/test_gpu_conj_sparse.py tests/test_gpu_configs.py > gpurun_out/r6_dfa_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r6_dfa_tests.log
[ $rc -ne 0 ] && exit $rc
STAMPS=1 timeout -k 10 400 python -u tools/ssb_host_times.py config4-scan > gpurun_out/r6_dfa_ssbh.txt 2> gpurun_out/r6_dfa_ssbh.err
rc=$?; echo "ssbh rc=$rc"; tail -15 gpurun_out/r6_dfa_ssbh.txt
exit $rc
