#!/bin/bash
# GPU-box job: RunOnce / scope / expansion / sweep parity tests, then the small legs' split
# (expansion on its own stream, verdict-only) and the sweep call's host split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_runonce.py tests/test_gpu_parity.py \
  tests/test_scope.py tests/test_gpu_planner.py -m gpu > gpurun_out/pytest_exp.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_exp.log
[[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; tail -60 gpurun_out/pytest_exp.log; exit $rc; }
timeout -k 10 300 python -u scripts/r6_legs_split.py > gpurun_out/legs_split.txt 2> gpurun_out/legs_split.err || { tail -20 gpurun_out/legs_split.err; exit 1; }
cat gpurun_out/legs_split.txt
CASIM_KNOBS=1 CASIM_DEBUG_TIMING=1 timeout -k 10 300 python -u scripts/r6_sweep_split.py > gpurun_out/swsplit_dbg.out 2> gpurun_out/swsplit_dbg.err || { tail -20 gpurun_out/swsplit_dbg.err; exit 1; }
cat gpurun_out/swsplit_dbg.out
grep "entry to core\|\] done" gpurun_out/swsplit_dbg.err | head -8
timeout -k 10 300 python -u scripts/runonce_diag.py > gpurun_out/rdiag.out 2> gpurun_out/rdiag.err || { tail -20 gpurun_out/rdiag.err; exit 1; }
cat gpurun_out/rdiag.out
