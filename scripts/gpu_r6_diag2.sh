#!/bin/bash
# GPU-box job: the RunOnce loop with the library's debug timing (expansion / sweep entry),
# and the chain's section cycles on C2 (CASIM_PROF build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/runonce_diag.py --phases > gpurun_out/rdiag.out 2> gpurun_out/rdiag.err || { tail -20 gpurun_out/rdiag.err; exit 1; }
cat gpurun_out/rdiag.out
grep "^\[expansion\]" gpurun_out/rdiag.err
CASIM_LIB_PATH=$PWD/autoscaler_amd/lib/libcasim_prof.so timeout -k 10 200 python -u scripts/chain_diag.py > gpurun_out/chain_diag.log 2>&1 || { tail gpurun_out/chain_diag.log; exit 1; }
cat gpurun_out/chain_diag.log
