#!/bin/bash
# (variant builds: make -C autoscaler_amd/csrc OUT=../lib/<name> BUILD=../../build/<name> "EXTRA=-DCASIM_PUB_BLOCKS_DECOUPLED=<N>")
# GPU-box job: the publisher's blocks with the decoupled Go order (64 / 256 against 128):
# Estimate parity tests on each variant, then the
# headline A/B (autoscaler_amd/lib/pb64, pb256).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in pb64 pb256; do
  CASIM_LIB_PATH=$PWD/autoscaler_amd/lib/$v/libcasim.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/pytest_$v.log 2>&1 \
    || { echo "TESTS FAILED $v"; tail -30 gpurun_out/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"
done
timeout -k 10 600 python -u scripts/ab_lib.py autoscaler_amd/lib/libcasim.so autoscaler_amd/lib/pb64/libcasim.so \
  autoscaler_amd/lib/pb256/libcasim.so 4 > gpurun_out/ab_pb.txt 2>&1; rc=$?
grep "median of medians" gpurun_out/ab_pb.txt
exit $rc
