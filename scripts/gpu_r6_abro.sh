#!/bin/bash
# GPU-box job: FilterOutSchedulable / RunOnce / sweep tests with the default build, then the
# C5 RunOnce legs A/B (scripts/ab_runonce.py) and the filter A/B (gpu_r6_abreplay.sh) of the
# default build against autoscaler_amd/lib/ab/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_filter.py tests/test_filter_out.py \
  tests/test_runonce.py tests/test_scope.py tests/test_gpu_parity.py -m gpu > gpurun_out/pytest_abro.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_abro.log
[[ $rc -eq 0 ]] || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_abro.log | head -80; exit $rc; }
timeout -k 10 900 python -u scripts/ab_runonce.py autoscaler_amd/lib/ab/libcasim.so autoscaler_amd/lib/libcasim.so 4 > gpurun_out/ab_runonce.txt 2>&1 \
  || { tail -20 gpurun_out/ab_runonce.txt; exit 1; }
cat gpurun_out/ab_runonce.txt
scripts/gpu_r6_abreplay.sh
