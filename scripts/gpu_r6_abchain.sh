#!/bin/bash
# GPU-box job: Estimate parity with the default build, then the headline A/B of the default
# build (autoscaler_amd/lib/libcasim.so) against a baseline build (autoscaler_amd/lib/ab/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multi.py \
  tests/test_scaleup.py tests/test_runonce.py tests/test_scope.py tests/test_gpu_shard.py -m gpu > gpurun_out/pytest_abchain.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_abchain.log
[[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; grep -B5 -A30 "Error\|assert" gpurun_out/pytest_abchain.log | head -100; exit $rc; }
timeout -k 10 600 python -u scripts/ab_lib.py autoscaler_amd/lib/ab/libcasim.so autoscaler_amd/lib/libcasim.so 4 > gpurun_out/ab_lib.txt 2>&1 || { tail -20 gpurun_out/ab_lib.txt; exit 1; }
cat gpurun_out/ab_lib.txt
