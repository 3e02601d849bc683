#!/bin/bash
# GPU-box job: podset creation timing, then the tests that build pod sets (parity, RunOnce, scope, multi).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/r6_podset_time.py > gpurun_out/podset.txt 2>&1 || { tail -20 gpurun_out/podset.txt; exit 1; }
cat gpurun_out/podset.txt
CASIM_KNOBS=1 CASIM_DEBUG_TIMING=1 timeout -k 10 300 python -u scripts/r6_podset_time.py > gpurun_out/podset_dbg.txt 2>&1 || { tail -20 gpurun_out/podset_dbg.txt; exit 1; }
grep "^\[podset\]" gpurun_out/podset_dbg.txt | tail -3
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_runonce.py tests/test_scope.py \
  tests/test_gpu_multi.py tests/test_gpu_filter.py tests/test_scaleup.py tests/test_c_abi.py -m gpu > gpurun_out/pytest_podset.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_podset.log
[[ $rc -eq 0 ]] || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_podset.log | head -80; exit $rc; }
