#!/bin/bash
# config-3 bench under several environment settings: each ENVS item is "NAME=VAL,NAME=VAL" (or "-" for none);
# one line per setting in gpurun_out/env_sweep.txt.
set -o pipefail
mkdir -p gpurun_out
for e in ${ENVS:--}; do
  envs=()
  [ "$e" != "-" ] && IFS=, read -ra envs <<< "$e"
  r=$(env "${envs[@]}" timeout -k 10 200 python3 bench.py --workload ${W:-config3} --steps 10 --warmup 2 --no-cpu \
      --no-parity 2>gpurun_out/env_sweep.err | python3 -c "import json,sys; d=json.load(sys.stdin); print('kernel_ms', round(d['roofline']['kernel_ms'],3), 'ms_per_step', round(d['ms_per_step'],3))") || { tail -5 gpurun_out/env_sweep.err; exit 1; }
  echo "$e $r" | tee -a gpurun_out/env_sweep.txt
done
