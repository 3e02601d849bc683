#!/bin/bash
# GPU-box job: the C5 RunOnce sweep at several host-walk look-ahead lengths (knob
# CASIM_SWEEP_LOOKAHEAD): rounds and leg time per loop.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for la in 512 1024 2048 4096 512; do
  CASIM_KNOBS=1 CASIM_SWEEP_LOOKAHEAD=$la timeout -k 10 300 python -u scripts/runonce_diag.py > gpurun_out/look_$la.out 2> gpurun_out/look_$la.err || { tail -20 gpurun_out/look_$la.err; exit 1; }
  echo "== lookahead $la"; grep -v "^filter" gpurun_out/look_$la.out | tail -4
done
