#!/bin/bash
# r6: per-query device time of both SSB flights with the sparse plans forced off (streaming kernels) vs the default
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for W in config4-scan config4; do
  for V in default off; do
    if [ $V = off ]; then export PH_GROUP_SPARSE=0 PH_AGG_SPARSE=0; else unset PH_GROUP_SPARSE PH_AGG_SPARSE; fi
    timeout -k 10 400 python -u tools/ssb_host_times.py $W > gpurun_out/r6s_${W}_$V.txt 2> gpurun_out/r6s_${W}_$V.err
    rc=$?; echo "$W $V rc=$rc"; [ $rc -ne 0 ] && exit $rc
    cat gpurun_out/r6s_${W}_$V.txt
  done
done
exit 0
