#!/bin/bash
# r3: new parity tests (hash-mode numGroupsLimit, filtered optimistic limit, k_part_reg widths), the SSB diagnostic,
# then the k_part_reg component sweep
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lean_widths.py tests/test_gpu_concurrency.py \
  -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_new.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_new.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/pytest_new.log | head -30; exit $rc; fi
timeout -k 10 300 python3 -u tools/diag_ssb.py > gpurun_out/diag_ssb.txt 2>&1; rc=$?; grep -E "ok=False|bad" gpurun_out/diag_ssb.txt | head -20
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r3f.sh
