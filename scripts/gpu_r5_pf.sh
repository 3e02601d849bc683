#!/bin/bash
# GPU-box job (round 5): planner parity, then the planner phase profile (prof build) and timing (release build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_planner.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_planner.log 2>&1 || { tail -30 gpurun_out/pytest_planner.log; exit 1; }
tail -2 gpurun_out/pytest_planner.log
timeout -k 10 200 python -u scripts/plan_prof.py --prof > gpurun_out/plan_prof.log 2>&1 || { tail -20 gpurun_out/plan_prof.log; exit 1; }
cat gpurun_out/plan_prof.log
timeout -k 10 200 python -u scripts/plan_prof.py > gpurun_out/plan_rel.log 2>&1 || { tail -20 gpurun_out/plan_rel.log; exit 1; }
grep -E "^limit|host:" gpurun_out/plan_rel.log
echo PF_OK
