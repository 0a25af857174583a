#!/bin/bash
# r3: full GPU suite (k_part_reg default, hash-mode numGroupsLimit, raw real predicates, 2-rank dense combine,
# FK_CONJ set-leaf fix), SSB 10M-row diagnostic, config4 bench (parity sample)
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 300 python3 -u tools/diag_ssb.py > gpurun_out/diag_ssb.txt 2>&1; rc=$?; grep -E "ok=False|bad" gpurun_out/diag_ssb.txt | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload config4 --steps 5 --warmup 2 --cpu-seconds 3 \
  > gpurun_out/bench_config4.json 2> gpurun_out/bench_config4.err
rc=$?; echo "bench config4 rc=$rc"; cat gpurun_out/bench_config4.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/sweep_inproc.py config3 "-" "PH_PART_DBG=2" "PH_PART_LDS=1" "-" > gpurun_out/r3_sweep_reg3.txt 2>&1
rc=$?; tail -5 gpurun_out/r3_sweep_reg3.txt; exit $rc
