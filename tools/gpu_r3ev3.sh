#!/bin/bash
# Round-3 evidence, part 3: rocprofv3 kernel-trace summaries (no counters) of every bench workload.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for w in ${PROF:-config3 config3-lds config2 config3-agg config4 config5}; do bash tools/gpu_prof.sh $w _r3 || exit $?; done
