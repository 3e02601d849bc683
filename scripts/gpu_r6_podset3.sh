#!/bin/bash
# GPU-box job: filter / RunOnce tests and timings with the staged pod-table uploads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_filter.py tests/test_filter_out.py tests/test_runonce.py \
  tests/test_scope.py tests/test_gpu_parity.py -m gpu > gpurun_out/pytest_podset3.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_podset3.log
[[ $rc -eq 0 ]] || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_podset3.log | head -80; exit $rc; }
timeout -k 10 300 python -u scripts/filter_timing.py c5 c5-c4 c5-loose > gpurun_out/ftime3.txt 2>&1 || { tail -20 gpurun_out/ftime3.txt; exit 1; }
cut -c1-60,200-260 gpurun_out/ftime3.txt
timeout -k 10 300 python -u scripts/runonce_diag.py > gpurun_out/rdiag3.out 2>&1 || { tail -20 gpurun_out/rdiag3.out; exit 1; }
grep "^{" gpurun_out/rdiag3.out
