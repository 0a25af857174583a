#!/bin/bash
# Round-5 iteration: the parity suites the changed kernels touch, then device times per workload.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_lean_widths.py tests/test_gpu_configs.py tests/test_gpu_conj_sparse.py tests/test_gpu_parity.py \
  > gpurun_out/iter_tests.log 2>&1 || { tail -40 gpurun_out/iter_tests.log; exit 1; }
tail -3 gpurun_out/iter_tests.log
for w in config3 config2 config3-lds config3-agg; do
  timeout -k 10 300 python3 -u tools/sweep_inproc.py $w "-" 2>&1 | grep device_ms || exit 1
done
timeout -k 10 400 python3 -u bench.py --workload config4-scan --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/c4s.json 2> gpurun_out/c4s.err || { tail -5 gpurun_out/c4s.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c4s.json')); print('config4-scan ms_per_step', round(d['ms_per_step'],2), 'kernel_ms', round(d['roofline']['kernel_ms'],2))"
timeout -k 10 400 python3 -u bench.py --workload config4 --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -5 gpurun_out/c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c4.json')); print('config4 ms_per_step', round(d['ms_per_step'],2), 'kernel_ms', round(d['roofline']['kernel_ms'],2))"
