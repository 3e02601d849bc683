#!/bin/bash
# GPU-box job (round 5): A/B of library variants (autoscaler_amd/lib/alt, alt2) against the
# default one on the planner: parity of each, then alternating release timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VARS="base"
for v in alt alt2; do [[ -f autoscaler_amd/lib/$v/libcasim.so ]] && VARS="$VARS $v"; done
lib() { [[ $1 == base ]] && echo "" || echo "autoscaler_amd/lib/$1/libcasim.so"; }
for v in $VARS; do
  if [[ $v == base ]]; then unset CASIM_LIB_PATH; else export CASIM_LIB_PATH=$(lib $v); fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_planner.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_planner_$v.log 2>&1 || { echo "PARITY FAILED $v"; tail -30 gpurun_out/pytest_planner_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pytest_planner_$v.log)"
done
unset CASIM_LIB_PATH
for rep in 1 2; do
  for v in $VARS; do
    if [[ $v == base ]]; then unset CASIM_LIB_PATH; else export CASIM_LIB_PATH=$(lib $v); fi
    timeout -k 10 200 python -u scripts/plan_host_split.py > gpurun_out/plan_split_$v.log 2>&1 || { tail -20 gpurun_out/plan_split_$v.log; exit 1; }
    echo "== $v"; cat gpurun_out/plan_split_$v.log
  done
done
echo AB_OK
