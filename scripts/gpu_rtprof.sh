#!/bin/bash
# GPU-box job: chain and run-table section cycles (CASIM_PROF build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
CASIM_LIB_PATH=$PWD/autoscaler_amd/lib/libcasim_prof.so timeout -k 10 200 python -u scripts/chain_diag.py > gpurun_out/chain_diag.log 2>&1 || { tail gpurun_out/chain_diag.log; exit 1; }
grep -A8 "k_run_table cycles" gpurun_out/chain_diag.log
echo RTPROF_OK
