#!/bin/bash
# GPU-box job: the -m gpu suite (optionally a -k filter as $1), log under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
K=${1:+-k "$1"}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $K > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || tail -60 gpurun_out/pytest_gpu.log
exit $rc
