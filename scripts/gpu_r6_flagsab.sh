#!/bin/bash
# GPU-box job: the C5 RunOnce sweep with and without the row-flag overlap (CASIM_SWEEP_SYNC_ROUNDS), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in flags sync flags sync flags sync; do
  if [[ $mode == sync ]]; then export CASIM_SWEEP_SYNC_ROUNDS=1; else unset CASIM_SWEEP_SYNC_ROUNDS; fi
  CASIM_KNOBS=1 timeout -k 10 300 python -u scripts/runonce_diag.py > gpurun_out/flags_$mode.out 2> gpurun_out/flags_$mode.err || { tail -20 gpurun_out/flags_$mode.err; exit 1; }
  echo "== $mode"; grep "^sweep\|^{" gpurun_out/flags_$mode.out | tail -4 | cut -c1-180
done
timeout -k 10 300 python -u scripts/sweep_timing.py > gpurun_out/sweep_c3.txt 2>&1 && tail -5 gpurun_out/sweep_c3.txt
