#!/bin/bash
# GPU-box job (round 5): A/B of planner variants — library builds (autoscaler_amd/lib/alt,
# alt2) and knob settings (h0: no helper waves) — against the default: parity of each, then
# alternating release timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VARS="base ${AB_KNOB_VARS:-}"
for v in alt alt2; do [[ -f autoscaler_amd/lib/$v/libcasim.so ]] && VARS="$VARS $v"; done
setv() {
  unset CASIM_LIB_PATH CASIM_KNOBS CASIM_PLAN_HELPERS
  case $1 in
    base) ;;
    h0) export CASIM_KNOBS=1 CASIM_PLAN_HELPERS=0 ;;
    h3) export CASIM_KNOBS=1 CASIM_PLAN_HELPERS=3 ;;
    *) export CASIM_LIB_PATH=autoscaler_amd/lib/$1/libcasim.so ;;
  esac
}
for v in $VARS; do
  setv $v
  timeout -k 10 300 python -u -m pytest tests/test_gpu_planner.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_planner_$v.log 2>&1 || { echo "PARITY FAILED $v"; tail -30 gpurun_out/pytest_planner_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pytest_planner_$v.log)"
done
for rep in 1 2; do
  for v in $VARS; do
    setv $v
    timeout -k 10 200 python -u scripts/plan_host_split.py > gpurun_out/plan_split_$v.log 2>&1 || { tail -20 gpurun_out/plan_split_$v.log; exit 1; }
    echo "== $v"; cat gpurun_out/plan_split_$v.log
  done
done
echo AB_OK
