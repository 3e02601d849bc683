#!/bin/bash
# (variant builds: make -C autoscaler_amd/csrc OUT=../lib/<name> BUILD=../../build/<name> "EXTRA=-DCASIM_SWEEP_WAVES=<N>" / "-DCASIM_PDQ_T_SMALL=<N>")
# GPU-box job: the C3 sweep A/B against 2 and 8 waves per EU for k_sweep (autoscaler_amd/lib/
# sw2, sw8; results digests compared), then the headline A/B against the Go-order sort's
# wavefront-phase frame bound at 512 and 2048 (autoscaler_amd/lib/ts512, ts2048).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/ab_sweep.py autoscaler_amd/lib/libcasim.so autoscaler_amd/lib/sw2/libcasim.so \
  autoscaler_amd/lib/sw8/libcasim.so 3 > gpurun_out/ab_sw.txt 2>&1; rc=$?
cat gpurun_out/ab_sw.txt
[[ $rc -eq 0 ]] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "estimate or headline or c2 or sort" \
  > gpurun_out/pytest_ts.log 2>&1 || true
timeout -k 10 600 python -u scripts/ab_lib.py autoscaler_amd/lib/libcasim.so autoscaler_amd/lib/ts512/libcasim.so \
  autoscaler_amd/lib/ts2048/libcasim.so 4 > gpurun_out/ab_ts.txt 2>&1; rc=$?
grep "median of medians" gpurun_out/ab_ts.txt
exit $rc
