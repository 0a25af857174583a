#!/bin/bash
# k_group_sparse container mode: its parity cases, then the inverted SSB flight with it (PH_GROUP_CONT=1) and without.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_configs.py \
  -k "group_sparse or config4" > gpurun_out/gcont_tests.log 2>&1 || { tail -30 gpurun_out/gcont_tests.log; exit 1; }
tail -2 gpurun_out/gcont_tests.log
for gc in 1 0; do
  PH_GROUP_CONT=$gc timeout -k 10 400 python3 -u bench.py --workload config4 --steps 5 --warmup 2 --no-cpu --no-parity \
    > gpurun_out/gcont_$gc.json 2> gpurun_out/gcont_$gc.err || { tail -5 gpurun_out/gcont_$gc.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/gcont_$gc.json')); print('PH_GROUP_CONT=$gc ms/step %.3f kernel_ms %.3f' % (d['ms_per_step'], d['roofline']['kernel_ms']))"
done
