#!/bin/bash
# (variant builds: make -C autoscaler_amd/csrc OUT=../lib/<name> BUILD=../../build/<name> "EXTRA=-DCASIM_PC_SKY=.. -DCASIM_PC_BULK_FAILS=.. -DCASIM_PC_BULK_SKIP=.. / -DCASIM_FB_BACKOFF=.. / -DCASIM_FB_ROWWISE_MAX=..")
# GPU-box job: planner A/B, second pass: the default build against 6- and 7-point block
# skylines and 6 points with the bulk back-off at 2/64 and 3/32 (autoscaler_amd/lib/{sky6,
# sky7,s6b2,s6b3}); results digests compared.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/ab_planner.py autoscaler_amd/lib/libcasim.so autoscaler_amd/lib/sky6/libcasim.so \
  autoscaler_amd/lib/sky7/libcasim.so autoscaler_amd/lib/s6b2/libcasim.so autoscaler_amd/lib/s6b3/libcasim.so --rounds 4 \
  > gpurun_out/ab_sky2.txt 2>&1; rc=$?
cat gpurun_out/ab_sky2.txt
exit $rc
