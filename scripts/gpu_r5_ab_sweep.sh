#!/bin/bash
# GPU-box job (round 5): A/B of library variants (autoscaler_amd/lib/alt, alt2) on the sweep:
# sweep / RunOnce / multi / planner parity of each variant, then C3 and C5 RunOnce sweep timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VARS="base"
for v in alt alt2; do [[ -f autoscaler_amd/lib/$v/libcasim.so ]] && VARS="$VARS $v"; done
setv() { unset CASIM_LIB_PATH; [[ $1 == base ]] || export CASIM_LIB_PATH=autoscaler_amd/lib/$1/libcasim.so; }
for v in $VARS; do
  [[ $v == base ]] && continue
  setv $v
  timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_runonce.py tests/test_gpu_multi.py tests/test_gpu_planner.py \
    -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_sweep_$v.log 2>&1 \
    || { echo "PARITY FAILED $v"; tail -30 gpurun_out/pytest_sweep_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pytest_sweep_$v.log)"
done
for rep in 1 2; do
  for v in $VARS; do
    setv $v
    timeout -k 10 200 python -u scripts/sweep_timing.py > gpurun_out/sw_$v.log 2>&1 || { tail -20 gpurun_out/sw_$v.log; exit 1; }
    timeout -k 10 200 python -u scripts/runonce_timing.py > gpurun_out/ro_$v.log 2>&1 || { tail -20 gpurun_out/ro_$v.log; exit 1; }
    echo "== $v"; grep -E "call_ms" gpurun_out/sw_$v.log; tail -3 gpurun_out/ro_$v.log
  done
done
echo ABS_OK
