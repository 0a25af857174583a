#!/bin/bash
# r3: batched statistics pass -- the filter-entry parity tests and the SSB configs
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_range_index.py \
  -m gpu -q --maxfail=5 --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ev7.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_ev7.log | tail -8; exit $rc
