#!/bin/bash
# GPU-box job: C3 sweep, C5 RunOnce sweep leg and the planner loop, the HEAD library
# (autoscaler_amd/lib/libcasim_head.so) against the working tree's.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for lib in libcasim_head.so libcasim.so; do
  echo "== $lib"
  export CASIM_LIB_PATH=$PWD/autoscaler_amd/lib/$lib
  timeout -k 10 120 python -u scripts/sweep_timing.py 5000 > gpurun_out/ab_$lib.log 2>&1 || { tail -5 gpurun_out/ab_$lib.log; exit 1; }
  grep -E "^fresh|^hinted call" gpurun_out/ab_$lib.log
  timeout -k 10 200 python -u scripts/planner_timing.py 5000 > gpurun_out/abp_$lib.log 2>&1 || { tail -5 gpurun_out/abp_$lib.log; exit 1; }
  cat gpurun_out/abp_$lib.log
  timeout -k 10 200 python -u scripts/runonce_diag.py > gpurun_out/abr_$lib.log 2>&1 || { tail -5 gpurun_out/abr_$lib.log; exit 1; }
  grep -v "^filter\|^sweep" gpurun_out/abr_$lib.log | tail -2
done
unset CASIM_LIB_PATH
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
exit $rc
