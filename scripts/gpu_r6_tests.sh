#!/bin/bash
# GPU-box job: selected GPU tests (the library is built here, in-tree, and travels).
# Usage: scripts/gpu_r6_tests.sh <pytest args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_sel.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_sel.log | tail -3
[[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; tail -60 gpurun_out/pytest_sel.log; exit $rc; }
