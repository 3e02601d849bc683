#!/bin/bash
# GPU-box job: expansion-plan tests, then the expansion call's host split inside the RunOnce
# loop (CASIM_DEBUG_TIMING) and alone (r6_legs_split.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_scaleup.py tests/test_runonce.py \
  -m gpu > gpurun_out/pytest_expsplit.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_expsplit.log
[[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; tail -60 gpurun_out/pytest_expsplit.log; exit $rc; }
CASIM_KNOBS=1 CASIM_DEBUG_TIMING=1 timeout -k 10 300 python -u scripts/runonce_diag.py > gpurun_out/rdiag.out 2> gpurun_out/rdiag.err || { tail -20 gpurun_out/rdiag.err; exit 1; }
grep "^{" gpurun_out/rdiag.out
grep "\[expansion\]" gpurun_out/rdiag.err
timeout -k 10 300 python -u scripts/r6_legs_split.py > gpurun_out/legs_split.txt 2> gpurun_out/legs_split.err || { tail -20 gpurun_out/legs_split.err; exit 1; }
cat gpurun_out/legs_split.txt
