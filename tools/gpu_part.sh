#!/bin/bash
# Partitioned group-by iteration on the GPU box: the parity tests of kernels A/B, then the config-3 device time in one
# process (tools/sweep_inproc.py; SWEEP_ROWS rows, default 1e9) under each setting given as arguments.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_lean_widths.py tests/test_gpu_configs.py::test_config3_headline_shape \
  "tests/test_gpu_parity.py::test_partition_multi_batch" "tests/test_gpu_parity.py::test_partition_overflow_skew" \
  "tests/test_gpu_parity.py::test_partition_wide_records" "tests/test_gpu_parity.py::test_partition_count_only_and_no_filter" \
  > gpurun_out/part_tests.log 2>&1 || { tail -30 gpurun_out/part_tests.log; exit 1; }
tail -3 gpurun_out/part_tests.log
[ -n "$NO_SWEEP" ] && exit 0
timeout -k 10 400 python3 -u tools/sweep_inproc.py ${W:-config3} "$@" 2>&1 | tee gpurun_out/part_sweep.txt
