#!/bin/bash
# (variant builds: make -C autoscaler_amd/csrc OUT=../lib/cw<N> BUILD=../../build/cw<N> "EXTRA=-DCASIM_CW=<N>")
# GPU-box job: headline A/B of the default build (4 waves per chain workgroup) against 2 and
# 8 waves (autoscaler_amd/lib/cw2, cw8), alternating processes, 40 steps each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/ab_lib.py autoscaler_amd/lib/libcasim.so autoscaler_amd/lib/cw2/libcasim.so \
  autoscaler_amd/lib/cw8/libcasim.so 4 > gpurun_out/ab_cw.txt 2>&1; rc=$?
cat gpurun_out/ab_cw.txt
exit $rc
