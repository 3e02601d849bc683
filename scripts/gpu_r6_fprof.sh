#!/bin/bash
# GPU-box job: FilterOutSchedulable cycle split (CASIM_PROF build) at C5 vs the loose regime.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/filter_timing.py --prof c5 c5-loose c5-loose-nohints > gpurun_out/fprof.txt 2>&1 || { tail -20 gpurun_out/fprof.txt; exit 1; }
timeout -k 10 300 python -u scripts/filter_timing.py --prof --bulk c5 c5-loose > gpurun_out/fprof_bulk.txt 2>&1 || { tail -20 gpurun_out/fprof_bulk.txt; exit 1; }
timeout -k 10 300 python -u scripts/filter_timing.py --phases c5 c5-loose > gpurun_out/fphases.txt 2>&1 || { tail -20 gpurun_out/fphases.txt; exit 1; }
cat gpurun_out/fprof.txt gpurun_out/fprof_bulk.txt
grep -v "^\[" gpurun_out/fphases.txt | head; grep "^\[filter" gpurun_out/fphases.txt | tail -30
timeout -k 10 300 python -u scripts/ab_head.py CASIM_SORT_FIRST 12 > gpurun_out/ab_sortfirst.txt 2>&1 || { tail -20 gpurun_out/ab_sortfirst.txt; exit 1; }
cat gpurun_out/ab_sortfirst.txt
