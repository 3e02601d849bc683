#!/bin/bash
# GPU-box job: sweep / RunOnce / multi / planner parity tests, then the C5 RunOnce sweep's
# per-round split (CASIM_DEBUG_TIMING) and the legs' timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_runonce.py tests/test_gpu_multi.py tests/test_gpu_shard.py tests/test_gpu_planner.py tests/test_c_abi.py -m gpu \
  > gpurun_out/pytest_sweep.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_sweep.log
[[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; tail -60 gpurun_out/pytest_sweep.log; exit $rc; }
timeout -k 10 300 python -u scripts/runonce_diag.py --phases > gpurun_out/rdiag.out 2> gpurun_out/rdiag.err || { tail -20 gpurun_out/rdiag.err; exit 1; }
cat gpurun_out/rdiag.out
grep "^\[sweep\]" gpurun_out/rdiag.err | tail -45
