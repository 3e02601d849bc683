#!/bin/bash
# GPU-box job: FilterOutSchedulable parity tests, then its timing (release and CASIM_PROF splits).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_filter.py tests/test_runonce.py tests/test_filter_out.py -m gpu > gpurun_out/pytest_filter.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_filter.log
[[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; tail -60 gpurun_out/pytest_filter.log; exit $rc; }
timeout -k 10 300 python -u scripts/filter_timing.py c5 c5-c4 c5-loose c5-loose-nohints c5-allhints > gpurun_out/ftime.txt 2>&1 || { tail -20 gpurun_out/ftime.txt; exit 1; }
cat gpurun_out/ftime.txt
timeout -k 10 300 python -u scripts/filter_timing.py --prof --bulk c5 c5-loose > gpurun_out/fprof_bulk2.txt 2>&1 || { tail -20 gpurun_out/fprof_bulk2.txt; exit 1; }
cat gpurun_out/fprof_bulk2.txt
