#!/bin/bash
# GPU-box job: the one-wave register chain (k_ffd_chain1) — Estimate parity tests, then the
# headline A/B against the four-wave LDS chain (CASIM_NO_REG_CHAIN) and the per-group times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_multi.py \
  tests/test_scaleup.py tests/test_runonce.py tests/test_gpu_shard.py tests/test_c_abi.py -m gpu > gpurun_out/pytest_chain1.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_chain1.log
[[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; grep -B5 -A40 "Error\|assert" gpurun_out/pytest_chain1.log | head -120; exit $rc; }
timeout -k 10 300 python -u scripts/ab_head.py CASIM_NO_REG_CHAIN 10 > gpurun_out/ab_chain1.txt 2>&1 || { tail -20 gpurun_out/ab_chain1.txt; exit 1; }
cat gpurun_out/ab_chain1.txt
timeout -k 10 200 python -u scripts/chain_diag.py > gpurun_out/chain1_diag.log 2>&1 || { tail gpurun_out/chain1_diag.log; exit 1; }
head -8 gpurun_out/chain1_diag.log
