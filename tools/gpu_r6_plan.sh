#!/bin/bash
# r6: host planning sub-phases (PH_HOST_TIMES) on config 5 (400 segments), config 3 and the SSB scan flight
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
for w in config5 config3; do
  PH_HOST_TIMES=1 timeout -k 10 400 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu --no-parity \
    > gpurun_out/r6p_$w.json 2> gpurun_out/r6p_$w.err
  rc=$?; echo "$w rc=$rc"; [ $rc -ne 0 ] && exit $rc
  grep "ph host" gpurun_out/r6p_$w.err | tail -20
done
STAMPS=1 timeout -k 10 400 python -u tools/ssb_host_times.py config4-scan > gpurun_out/r6p_ssb.txt 2> gpurun_out/r6p_ssb.err
rc=$?; echo "ssb rc=$rc"; tail -2 gpurun_out/r6p_ssb.txt
exit $rc
