#!/bin/bash
# GPU-box job (round 5): A/B of a library variant (autoscaler_amd/lib/alt) on the sweep:
# sweep / RunOnce / planner parity of the variant, then C3 and C5 RunOnce sweep timings of both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ALT=autoscaler_amd/lib/alt/libcasim.so
CASIM_LIB_PATH=$ALT timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_runonce.py tests/test_gpu_multi.py tests/test_gpu_planner.py \
  -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_sweep_alt.log 2>&1 \
  || { echo "PARITY FAILED"; tail -30 gpurun_out/pytest_sweep_alt.log; exit 1; }
tail -1 gpurun_out/pytest_sweep_alt.log
for v in base alt base alt; do
  if [[ $v == alt ]]; then export CASIM_LIB_PATH=$ALT; else unset CASIM_LIB_PATH; fi
  timeout -k 10 200 python -u scripts/sweep_timing.py > gpurun_out/sw_$v.log 2>&1 || { tail -20 gpurun_out/sw_$v.log; exit 1; }
  timeout -k 10 200 python -u scripts/runonce_timing.py > gpurun_out/ro_$v.log 2>&1 || { tail -20 gpurun_out/ro_$v.log; exit 1; }
  echo "== $v"; grep -E "call_ms" gpurun_out/sw_$v.log; tail -2 gpurun_out/ro_$v.log
done
echo ABS_OK
