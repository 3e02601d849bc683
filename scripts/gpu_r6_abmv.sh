#!/bin/bash
# (variant builds: make -C autoscaler_amd/csrc OUT=../lib/mv<N> BUILD=../../build/mv<N> "EXTRA=-DCASIM_PC_MVBUF=<N>")
# GPU-box job: planner A/B of the default build (512 committed moves staged in LDS between
# flushes) against 1024 and 2048 (autoscaler_amd/lib/mv1024, mv2048); results digests compared.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/ab_planner.py autoscaler_amd/lib/libcasim.so autoscaler_amd/lib/mv1024/libcasim.so \
  autoscaler_amd/lib/mv2048/libcasim.so --rounds 4 > gpurun_out/ab_mv.txt 2>&1; rc=$?
cat gpurun_out/ab_mv.txt
[[ $rc -eq 0 ]] || exit $rc
# (and the sweep's look-ahead rows per table round: 256 / 384 / 768 against 512, RunOnce legs;
#  variant builds OUT=../lib/la<N> "EXTRA=-DCASIM_SWEEP_LOOKAHEAD_ROWS=<N>")
timeout -k 10 900 python -u scripts/ab_runonce.py autoscaler_amd/lib/libcasim.so autoscaler_amd/lib/la256/libcasim.so \
  autoscaler_amd/lib/la384/libcasim.so autoscaler_amd/lib/la768/libcasim.so 4 > gpurun_out/ab_la.txt 2>&1; rc=$?
grep median gpurun_out/ab_la.txt
exit $rc
