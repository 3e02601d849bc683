#!/bin/bash
# (variant builds: make -C autoscaler_amd/csrc OUT=../lib/<name> BUILD=../../build/<name> "EXTRA=-DCASIM_PCH_DECOUPLED=<N>")
# GPU-box job: the publisher's chunk with the decoupled Go order (32768 / 65536 against 16384):
# Estimate parity tests on each variant, then the
# headline A/B (autoscaler_amd/lib/pc16384, pc32768, pc65536).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in pc32768 pc65536; do
  CASIM_LIB_PATH=$PWD/autoscaler_amd/lib/$v/libcasim.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests/test_gpu_parity.py -m gpu > gpurun_out/pytest_$v.log 2>&1 \
    || { echo "TESTS FAILED $v"; tail -30 gpurun_out/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"
done
timeout -k 10 600 python -u scripts/ab_lib.py autoscaler_amd/lib/pc16384/libcasim.so autoscaler_amd/lib/pc32768/libcasim.so \
  autoscaler_amd/lib/pc65536/libcasim.so 4 > gpurun_out/ab_pch2.txt 2>&1; rc=$?
grep "median of medians" gpurun_out/ab_pch2.txt
exit $rc
