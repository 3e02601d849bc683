#!/bin/bash
# (variant builds: make -C autoscaler_amd/csrc OUT=../lib/<name> BUILD=../../build/<name> "EXTRA=-DCASIM_PC_SKY=.. -DCASIM_PC_BULK_FAILS=.. -DCASIM_PC_BULK_SKIP=.. / -DCASIM_FB_BACKOFF=.. / -DCASIM_FB_ROWWISE_MAX=..")
# GPU-box job: planner A/B of the default build against 6- and 4-point block skylines and the bulk back-off at 2/64 and 8/8
# (CASIM_PC_SKY / CASIM_PC_BULK_* builds under autoscaler_amd/lib/sky6, sky4, bk2, bk8), results digests compared.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/ab_planner.py autoscaler_amd/lib/libcasim.so autoscaler_amd/lib/sky6/libcasim.so \
  autoscaler_amd/lib/sky4/libcasim.so autoscaler_amd/lib/bk2/libcasim.so autoscaler_amd/lib/bk8/libcasim.so --rounds 3 > gpurun_out/ab_sky.txt 2>&1; rc=$?
cat gpurun_out/ab_sky.txt
exit $rc
