#!/bin/bash
# DFA chunk-size sweep on the scan-dimension SSB flight: AND-walk parity, then per-query wall times and a kernel trace
# per PH_DFA_CW setting (k_and_dfa's average duration in gpurun_out/dfa_cw<N>/run_kernel_stats.csv).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
export PYTHONUNBUFFERED=1 FLIGHT_NO_INVERTED=1
[ -n "$NO_TESTS" ] || timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_and_walk.py \
  > $ROOT/gpurun_out/dfa_tests.log 2>&1 || { tail -30 $ROOT/gpurun_out/dfa_tests.log; exit 1; }
tail -2 $ROOT/gpurun_out/dfa_tests.log
export TMPDIR=/tmp
for cw in ${CWS:-8 4 2}; do
  echo "== PH_DFA_CW=$cw"
  cd /tmp
  PH_DFA_CW=$cw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/dfa_cw$cw -o run -- \
    python3 $ROOT/tools/flight_times.py 60 4 > $ROOT/gpurun_out/dfa_cw$cw.txt 2>&1 || { tail -5 $ROOT/gpurun_out/dfa_cw$cw.txt; exit 1; }
  grep -E "^Q" $ROOT/gpurun_out/dfa_cw$cw.txt
  f=$(find $ROOT/gpurun_out/dfa_cw$cw -name "*kernel_stats.csv" | head -1)
  grep -E "k_and_dfa|k_and_compose" $f | cut -c1-160
done
if [ -n "$HOST_TIMES" ]; then
  cd $ROOT
  FLIGHT_ONLY=$HOST_TIMES PH_HOST_TIMES=1 timeout -k 10 300 python3 -u tools/flight_times.py 60 4 > gpurun_out/dfa_host.txt 2>&1 || exit 1
  tail -40 gpurun_out/dfa_host.txt
fi
