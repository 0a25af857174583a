#!/bin/bash
# r6: per-query wall / device / host split of both SSB flights, with the library's phase stamps (PH_HOST_TIMES)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for W in config4-scan config4; do
  STAMPS=1 timeout -k 10 400 python -u tools/ssb_host_times.py $W > gpurun_out/r6_ssbh_$W.txt 2> gpurun_out/r6_ssbh_$W.err
  rc=$?; echo "$W rc=$rc"; tail -15 gpurun_out/r6_ssbh_$W.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
