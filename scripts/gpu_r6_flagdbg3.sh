#!/bin/bash
# GPU-box job: the row-flag failure with the serial chain off, and with the debug output of
# the failing case.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T="tests/test_gpu_parity.py tests/test_runonce.py tests/test_gpu_multi.py tests/test_gpu_shard.py tests/test_gpu_planner.py"
CASIM_KNOBS=1 CASIM_NO_SERIAL_CHAIN=1 timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread $T -m gpu -k "planner" > gpurun_out/flagdbg3_nochain.log 2>&1; echo "no serial chain rc=$?"; tail -3 gpurun_out/flagdbg3_nochain.log
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_planner.py -m gpu > gpurun_out/flagdbg3_planner.log 2>&1; echo "planner file alone rc=$?"; tail -3 gpurun_out/flagdbg3_planner.log
