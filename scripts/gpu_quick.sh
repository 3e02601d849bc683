#!/bin/bash
# GPU-box job: GPU tests, then the planner and sweep timing scripts.  Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -u scripts/planner_timing.py 5000 > gpurun_out/planner_timing.log 2>&1 || { tail -20 gpurun_out/planner_timing.log; exit 1; }
cat gpurun_out/planner_timing.log
CASIM_DEBUG_TIMING=1 timeout -k 10 120 python -u scripts/planner_debug.py 5000 0 > gpurun_out/plan_dbg.log 2>&1 || { tail -20 gpurun_out/plan_dbg.log; exit 1; }
tail -2 gpurun_out/plan_dbg.log
