#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_planner.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_planner.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_planner.log; [[ $rc -eq 0 ]] || { tail -30 gpurun_out/pytest_planner.log; exit 1; }
timeout -k 10 200 python -u scripts/plan_prof.py 5000 > gpurun_out/plan_prof.log 2>&1 || { tail -20 gpurun_out/plan_prof.log; exit 1; }
grep -E "^limit|host:" gpurun_out/plan_prof.log
timeout -k 10 200 python -u scripts/plan_prof.py 5000 --prof > gpurun_out/plan_prof_p.log 2>&1 || { tail -20 gpurun_out/plan_prof_p.log; exit 1; }
grep -E "^limit|phases|plain" gpurun_out/plan_prof_p.log
echo PP_OK
