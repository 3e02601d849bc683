#!/bin/bash
# GPU-box job: C3 sweep timing, the HEAD library against the working tree's, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for r in 1 2; do
  for lib in libcasim_head.so libcasim.so; do
    echo "== $lib"
    CASIM_LIB_PATH=$PWD/autoscaler_amd/lib/$lib timeout -k 10 120 python -u scripts/sweep_timing.py 5000 > gpurun_out/ab_$lib.log 2>&1 || { tail -5 gpurun_out/ab_$lib.log; exit 1; }
    grep -E "^fresh|^hinted call" gpurun_out/ab_$lib.log
  done
done
CASIM_DEBUG_TIMING=1 timeout -k 10 120 python -u scripts/planner_debug.py 5000 0 > gpurun_out/plan_dbg.log 2>&1 || { tail -5 gpurun_out/plan_dbg.log; exit 1; }
tail -1 gpurun_out/plan_dbg.log
