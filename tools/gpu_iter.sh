#!/bin/bash
# One iteration on the GPU box: parity suite (stop on failure), then a kernel-trace profile per workload
# (config3 once more with PH_PART_SERIAL=1 so kernels A and B are timed without overlap).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
for w in ${WORKLOADS:-config2 config3}; do
  bash tools/gpu_prof.sh $w || exit $?
done
if [ -z "$NO_SERIAL" ]; then PH_PART_SERIAL=1 bash tools/gpu_prof.sh config3 serial || exit $?; fi
