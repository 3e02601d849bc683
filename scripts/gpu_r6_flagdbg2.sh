#!/bin/bash
# GPU-box job: the sweep / planner GPU tests in one process, without then with the row flags.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="tests/test_gpu_parity.py tests/test_runonce.py tests/test_gpu_multi.py tests/test_gpu_shard.py tests/test_gpu_planner.py"
CASIM_KNOBS=1 CASIM_SWEEP_SYNC_ROUNDS=1 timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread $T -m gpu > gpurun_out/flagdbg2_sync.log 2>&1; echo "sync rounds rc=$?"; tail -4 gpurun_out/flagdbg2_sync.log
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread $T -m gpu > gpurun_out/flagdbg2_flags.log 2>&1; echo "flags rc=$?"; tail -6 gpurun_out/flagdbg2_flags.log
