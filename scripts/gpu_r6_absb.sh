#!/bin/bash
# (variant builds: make -C autoscaler_amd/csrc OUT=../lib/sb<N> BUILD=../../build/sb<N> "EXTRA=-DCASIM_SIDE_BAND=<N>")
# GPU-box job: C5 RunOnce legs A/B of the default build against the sweep's side-row band
# at 16 and 32 classes (autoscaler_amd/lib/sb16, sb32).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/ab_runonce.py autoscaler_amd/lib/libcasim.so autoscaler_amd/lib/sb16/libcasim.so \
  autoscaler_amd/lib/sb32/libcasim.so 4 > gpurun_out/ab_sb.txt 2>&1; rc=$?
cat gpurun_out/ab_sb.txt
exit $rc
