#!/bin/bash
# r6: config-3 knob sweep in one process (device ms of A + B per setting), settings as arguments
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
W=${W:-config3}
timeout -k 10 ${T:-500} python3 -u tools/sweep_inproc.py $W "$@" > gpurun_out/r6_sweep_$W.txt 2>&1
rc=$?; cat gpurun_out/r6_sweep_$W.txt; exit $rc
