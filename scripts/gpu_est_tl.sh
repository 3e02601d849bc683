#!/bin/bash
# GPU-box job: Estimate parity tests, the headline bench alone, then a kernel trace of it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash scripts/gpu_est.sh || exit $?
bash scripts/gpu_tl.sh || exit $?
echo EST_TL_OK
