#!/bin/bash
# GPU-box job: the device sort's phase and per-step cycle counters (CASIM_PROF build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
CASIM_LIB_PATH=$PWD/autoscaler_amd/lib/libcasim_prof.so timeout -k 10 200 python -u scripts/pdq_prof.py > gpurun_out/pdq_prof.log 2>&1 || { tail gpurun_out/pdq_prof.log; exit 1; }
cat gpurun_out/pdq_prof.log
echo PDQ_OK
