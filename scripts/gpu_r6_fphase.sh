#!/bin/bash
# GPU-box job: FilterOutSchedulable host phases (CASIM_DEBUG_TIMING) in the loose and C5 regimes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/filter_timing.py --phases c5-loose > gpurun_out/fphase.txt 2> gpurun_out/fphase.err || { tail -20 gpurun_out/fphase.err; exit 1; }
cat gpurun_out/fphase.txt
tail -60 gpurun_out/fphase.err
