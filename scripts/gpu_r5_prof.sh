#!/bin/bash
# GPU-box job (round 5): planner phase profile (CASIM_PROF build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/plan_prof.py 5000 --prof > gpurun_out/plan_prof_p.log 2>&1 || { tail -20 gpurun_out/plan_prof_p.log; exit 1; }
cat gpurun_out/plan_prof_p.log
CASIM_PLAN_HELPERS=0 timeout -k 10 200 python -u scripts/plan_prof.py 5000 --prof > gpurun_out/plan_prof_p0.log 2>&1 || { tail -20 gpurun_out/plan_prof_p0.log; exit 1; }
cat gpurun_out/plan_prof_p0.log
echo PROF_OK
