#!/bin/bash
# GPU-box job (round 5): planner parity tests, then the planner's timings and phase profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_planner.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_planner.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_planner.log
[[ $rc -eq 0 ]] || { tail -40 gpurun_out/pytest_planner.log; exit $rc; }
timeout -k 10 200 python -u scripts/plan_prof.py 5000 > gpurun_out/plan_prof.log 2>&1 || { tail -20 gpurun_out/plan_prof.log; exit 1; }
cat gpurun_out/plan_prof.log
timeout -k 10 200 python -u scripts/plan_prof.py 5000 --prof > gpurun_out/plan_prof_p.log 2>&1 || { tail -20 gpurun_out/plan_prof_p.log; exit 1; }
cat gpurun_out/plan_prof_p.log
echo PLANNER_OK
