#!/bin/bash
# GPU-box job: the failing planner case with and without the row-flag overlap.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CASIM_KNOBS=1 CASIM_SWEEP_SYNC_ROUNDS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_planner.py -m gpu -k "test_plan_c3" > gpurun_out/flagdbg_sync.log 2>&1; echo "sync rounds rc=$?"; tail -2 gpurun_out/flagdbg_sync.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_planner.py -m gpu -k "test_plan_c3" > gpurun_out/flagdbg_flags.log 2>&1; echo "flags rc=$?"; tail -2 gpurun_out/flagdbg_flags.log
