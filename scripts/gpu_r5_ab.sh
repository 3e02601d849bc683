#!/bin/bash
# GPU-box job (round 5): A/B of a library variant (autoscaler_amd/lib/alt) against the
# default one on the planner: parity of both, then alternating release timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ALT=autoscaler_amd/lib/alt/libcasim.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_planner.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_planner.log 2>&1 || { tail -30 gpurun_out/pytest_planner.log; exit 1; }
tail -1 gpurun_out/pytest_planner.log
CASIM_LIB_PATH=$ALT timeout -k 10 300 python -u -m pytest tests/test_gpu_planner.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_planner_alt.log 2>&1 || { tail -30 gpurun_out/pytest_planner_alt.log; exit 1; }
tail -1 gpurun_out/pytest_planner_alt.log
for v in base alt base alt; do
  if [[ $v == alt ]]; then export CASIM_LIB_PATH=$ALT; else unset CASIM_LIB_PATH; fi
  timeout -k 10 200 python -u scripts/plan_host_split.py > gpurun_out/plan_split_$v.log 2>&1 || { tail -20 gpurun_out/plan_split_$v.log; exit 1; }
  echo "== $v"; cat gpurun_out/plan_split_$v.log
done
unset CASIM_LIB_PATH
CASIM_DEBUG_TIMING=1 timeout -k 10 200 python -u scripts/plan_host_split.py > gpurun_out/plan_split_dbg.log 2>&1 || { tail -20 gpurun_out/plan_split_dbg.log; exit 1; }
grep -E "^limit|\[plan chain|\[replay" gpurun_out/plan_split_dbg.log | tail -24
echo AB_OK
