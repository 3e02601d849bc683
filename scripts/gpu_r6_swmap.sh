#!/bin/bash
# GPU-box job: sweep / planner / multi-device / RunOnce tests, then the C5 sweep call's
# split (scripts/r6_sweep_split.py) plain and with CASIM_DEBUG_TIMING (table rounds: launch
# vs completion).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_planner.py \
  tests/test_gpu_multi.py tests/test_gpu_shard.py tests/test_scope.py tests/test_runonce.py -m gpu > gpurun_out/pytest_swmap.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_swmap.log
[[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; grep -B5 -A30 "Error\|assert" gpurun_out/pytest_swmap.log | head -80; exit $rc; }
timeout -k 10 300 python -u scripts/r6_sweep_split.py > gpurun_out/swsplit.out 2> gpurun_out/swsplit.err || { tail -20 gpurun_out/swsplit.err; exit 1; }
cat gpurun_out/swsplit.out
CASIM_KNOBS=1 CASIM_DEBUG_TIMING=1 timeout -k 10 300 python -u scripts/r6_sweep_split.py > gpurun_out/swsplit_dbg.out 2> gpurun_out/swsplit_dbg.err || { tail -20 gpurun_out/swsplit_dbg.err; exit 1; }
grep "re-centre\|table launched\|table sync\|table round" gpurun_out/swsplit_dbg.err | tail -16
