#!/bin/bash
# Round-2 evidence in one GPU call: full -m gpu suite, smoke, bench lines for every workload, kernel-trace profiles
# and PMC traffic for the headline (config3) and config5.  Stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
WORKLOADS=${WORKLOADS:-"config3 config2 config3-agg config3-lds config1 config5 config4"} CPU_SECS=${CPU_SECS:-5} \
  bash tools/gpu_check.sh || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
for w in ${PROF:-config3 config5 config2 config4}; do bash tools/gpu_prof.sh $w || exit $?; done
for w in ${PMC:-config3 config5}; do bash tools/gpu_pmc.sh $w || exit $?; done
