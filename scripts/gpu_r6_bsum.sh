#!/bin/bash
# GPU-box job: sweep parity with the table kernel's block summaries in LDS, then the C5 RunOnce
# sweep and the C3 sweep with and without (CASIM_SWEEP_BSUM_GLOBAL), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="tests/test_gpu_parity.py tests/test_runonce.py tests/test_gpu_multi.py tests/test_gpu_shard.py tests/test_gpu_planner.py tests/test_scope.py"
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread $T -m gpu > gpurun_out/pytest_bsum.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_bsum.log
[[ $rc -eq 0 ]] || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_bsum.log | head -80; exit $rc; }
for mode in lds glob lds glob; do
  if [[ $mode == glob ]]; then export CASIM_SWEEP_BSUM_GLOBAL=1; else unset CASIM_SWEEP_BSUM_GLOBAL; fi
  CASIM_KNOBS=1 timeout -k 10 300 python -u scripts/runonce_diag.py > gpurun_out/bsum_$mode.out 2> gpurun_out/bsum_$mode.err || { tail -20 gpurun_out/bsum_$mode.err; exit 1; }
  echo "== $mode"; grep "^sweep\|^{" gpurun_out/bsum_$mode.out | tail -2 | cut -c1-180
  CASIM_KNOBS=1 timeout -k 10 300 python -u scripts/sweep_timing.py > gpurun_out/bsum_c3_$mode.txt 2>&1 && grep "call_ms" gpurun_out/bsum_c3_$mode.txt | head -2
done
