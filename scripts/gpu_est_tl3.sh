#!/bin/bash
# GPU-box job: Estimate parity tests, the headline bench alone, a rocprofv3 kernel trace of
# a few headline steps (gpurun_out/tl.txt), the chain section cycles (CASIM_PROF build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash scripts/gpu_est.sh || exit 1
bash scripts/gpu_tl.sh || exit 1
CASIM_LIB_PATH=$PWD/autoscaler_amd/lib/libcasim_prof.so timeout -k 10 200 python -u scripts/chain_diag.py > gpurun_out/chain_diag.log 2>&1 || { tail gpurun_out/chain_diag.log; exit 1; }
cat gpurun_out/chain_diag.log
CASIM_LIB_PATH=$PWD/autoscaler_amd/lib/libcasim_prof.so timeout -k 10 200 python -u scripts/pdq_prof.py > gpurun_out/pdq_prof.log 2>&1 || { tail gpurun_out/pdq_prof.log; exit 1; }
cat gpurun_out/pdq_prof.log
echo EST_TL3_OK
