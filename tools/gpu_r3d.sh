#!/bin/bash
# r3: k_part_reg (register-direct kernel A) -- full GPU suite, SSB 10M-row parity diagnostic, config3 / config5 bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_lean_widths.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_part.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_part.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/pytest_part.log | head -30; exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 300 python3 -u tools/diag_ssb.py > gpurun_out/diag_ssb.txt 2>&1; rc=$?; grep -E "ok=False|bad|first" gpurun_out/diag_ssb.txt | head -20
[ $rc -eq 0 ] || exit $rc
for w in config3 config5; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 5 --warmup 2 --cpu-seconds 3 \
    > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err
  rc=$?; echo "bench $w rc=$rc"; cat gpurun_out/bench_$w.json
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/bench_$w.err; exit $rc; fi
done
