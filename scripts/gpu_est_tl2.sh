#!/bin/bash
# GPU-box job: Estimate parity tests, the headline bench alone, then a rocprofv3 kernel
# trace of a few headline steps (timeline in gpurun_out/tl.txt)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash scripts/gpu_est.sh || exit 1
bash scripts/gpu_tl.sh || exit 1
echo EST_TL_OK
