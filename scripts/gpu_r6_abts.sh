#!/bin/bash
# (variant builds: make -C autoscaler_amd/csrc OUT=../lib/ts<N> BUILD=../../build/ts<N> "EXTRA=-DCASIM_PDQ_T_SMALL=<N>")
# GPU-box job: Estimate parity tests (Go order included) on the Go-order sort's wavefront-
# phase frame bound at 2048 and 4096 (autoscaler_amd/lib/ts2048, ts4096), then the headline
# A/B of the default build (1024) against both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 2048 4096; do
  CASIM_LIB_PATH=$PWD/autoscaler_amd/lib/ts$v/libcasim.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_shard.py -m gpu > gpurun_out/pytest_ts$v.log 2>&1 \
    || { echo "TESTS FAILED ts$v"; tail -30 gpurun_out/pytest_ts$v.log; exit 1; }
  echo "ts$v: $(tail -1 gpurun_out/pytest_ts$v.log)"
done
timeout -k 10 600 python -u scripts/ab_lib.py autoscaler_amd/lib/libcasim.so autoscaler_amd/lib/ts2048/libcasim.so \
  autoscaler_amd/lib/ts4096/libcasim.so 4 > gpurun_out/ab_ts2.txt 2>&1; rc=$?
grep "median of medians" gpurun_out/ab_ts2.txt
exit $rc
