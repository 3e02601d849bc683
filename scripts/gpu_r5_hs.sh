#!/bin/bash
# GPU-box job (round 5): planner parity, then the host-side split of a planner call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_planner.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_planner.log 2>&1 || { tail -30 gpurun_out/pytest_planner.log; exit 1; }
tail -2 gpurun_out/pytest_planner.log
timeout -k 10 200 python -u scripts/plan_host_split.py > gpurun_out/plan_split.log 2>&1 || { tail -20 gpurun_out/plan_split.log; exit 1; }
cat gpurun_out/plan_split.log
CASIM_DEBUG_TIMING=1 timeout -k 10 200 python -u scripts/plan_host_split.py > gpurun_out/plan_split_dbg.log 2>&1 || { tail -20 gpurun_out/plan_split_dbg.log; exit 1; }
grep -E "^limit|\[plan" gpurun_out/plan_split_dbg.log | tail -40
timeout -k 10 200 python -u scripts/plan_prof.py > gpurun_out/plan_rel.log 2>&1 || { tail -20 gpurun_out/plan_rel.log; exit 1; }
grep -E "^limit|host:" gpurun_out/plan_rel.log
echo HS_OK
