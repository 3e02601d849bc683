#!/bin/bash
# GPU-box job: FilterOutSchedulable walk profile (CASIM_PROF build) and the C5 RunOnce legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/filter_timing.py --prof c5 c5-loose-nohints > gpurun_out/filter_prof.log 2>&1 || { tail -20 gpurun_out/filter_prof.log; exit 1; }
timeout -k 10 200 python -u scripts/filter_timing.py --prof --bulk c5 c5-loose-nohints > gpurun_out/filter_prof_bulk.log 2>&1 || { tail -20 gpurun_out/filter_prof_bulk.log; exit 1; }
grep -v "^\[" gpurun_out/filter_prof.log gpurun_out/filter_prof_bulk.log
timeout -k 10 300 python -u scripts/runonce_diag.py > gpurun_out/runonce_diag.log 2>&1 || { tail -20 gpurun_out/runonce_diag.log; exit 1; }
cat gpurun_out/runonce_diag.log
echo LEGS_OK
