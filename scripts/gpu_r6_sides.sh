#!/bin/bash
# GPU-box job: C5 RunOnce sweep with side rows for re-centred rows (knob
# CASIM_SWEEP_RECENTRE_SIDES) at two look-aheads: rounds and the library's sweep time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "0 512" "3 512" "3 256" "0 512" "3 512" "3 1024"; do
  set -- $cfg
  CASIM_KNOBS=1 CASIM_SWEEP_RECENTRE_SIDES=$1 CASIM_SWEEP_LOOKAHEAD=$2 timeout -k 10 300 python -u scripts/runonce_diag.py > gpurun_out/sides_$1_$2.out 2> gpurun_out/sides_$1_$2.err || { tail -20 gpurun_out/sides_$1_$2.err; exit 1; }
  echo "== sides $1 lookahead $2"; grep "^sweep\|^{" gpurun_out/sides_$1_$2.out | tail -4 | cut -c1-200
done
