#!/bin/bash
# Round-5 kernel-trace summaries of every workload, the SQ counters of config 3's kernels (k_part_reg / k_part_agg),
# and the one-process multi-device line (--devices 0,0).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out
PHASE=prof PROF="${PROF:-config3 config2 config3-agg config3-lds config1 config5 config4 config4-scan}" bash tools/gpu_r5final.sh || exit 1
W=config3 bash tools/gpu_kprof.sh - > gpurun_out/r5_kprof_config3.txt 2>&1 || { tail -5 gpurun_out/r5_kprof_config3.txt; exit 1; }
python3 tools/sq_summary.py gpurun_out/kprof_config3 > gpurun_out/r5_sq_config3.txt 2>&1
head -40 gpurun_out/r5_sq_config3.txt
PHASE=multi bash tools/gpu_r5final.sh
