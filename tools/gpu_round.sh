#!/bin/bash
# One GPU call: parity suite + smoke + bench lines, kernel-trace profile and PMC traffic of the headline workload.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
WORKLOADS=${WORKLOADS:-"config2 config3"} bash tools/gpu_check.sh || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
for w in ${PROF:-config3 config2}; do bash tools/gpu_prof.sh $w || exit $?; done
for w in ${PMC:-config3 config2}; do (cd $ROOT && bash tools/gpu_pmc.sh $w) || exit $?; cat gpurun_out/pmc_$w.json; done
