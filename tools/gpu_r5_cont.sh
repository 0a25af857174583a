#!/bin/bash
# Container-mode sparse kernels: their parity suites, then PMC + bench lines of the workloads they serve.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_conj_sparse.py \
  > gpurun_out/cont_tests.log 2>&1 || { tail -30 gpurun_out/cont_tests.log; exit 1; }
tail -2 gpurun_out/cont_tests.log
PHASE=pmc PMC="${PMC:-config5 config4 config4-scan}" bash tools/gpu_r5final.sh || exit 1
PHASE=bench BENCH="${BENCH:-config5 config4 config4-scan}" bash tools/gpu_r5final.sh
