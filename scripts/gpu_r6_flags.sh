#!/bin/bash
# GPU-box job: sweep parity with the row-flag host walk, then the C5 RunOnce sweep with and
# without it (CASIM_SWEEP_SYNC_ROUNDS), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_runonce.py \
  tests/test_gpu_multi.py tests/test_gpu_shard.py tests/test_gpu_planner.py tests/test_scope.py -m gpu > gpurun_out/pytest_flags.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_flags.log
[[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; grep -B5 -A30 "Error\|assert" gpurun_out/pytest_flags.log | head -100; exit $rc; }
for mode in flags sync flags sync; do
  if [[ $mode == sync ]]; then export CASIM_SWEEP_SYNC_ROUNDS=1; else unset CASIM_SWEEP_SYNC_ROUNDS; fi
  CASIM_KNOBS=1 timeout -k 10 300 python -u scripts/runonce_diag.py > gpurun_out/flags_$mode.out 2> gpurun_out/flags_$mode.err || { tail -20 gpurun_out/flags_$mode.err; exit 1; }
  echo "== $mode"; grep "^sweep\|^{" gpurun_out/flags_$mode.out | tail -4 | cut -c1-180
done
