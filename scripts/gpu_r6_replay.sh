#!/bin/bash
# GPU-box job: FilterOutSchedulable / RunOnce / planner tests with the bucketed AddPod replay,
# then the filter's host phases (CASIM_DEBUG_TIMING) and the RunOnce loop.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_filter.py tests/test_filter_out.py tests/test_runonce.py \
  tests/test_scope.py tests/test_gpu_planner.py tests/test_gpu_multi.py -m gpu > gpurun_out/pytest_replay.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_replay.log
[[ $rc -eq 0 ]] || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_replay.log | head -80; exit $rc; }
timeout -k 10 300 python -u scripts/filter_timing.py --phases c5 > gpurun_out/freplay.txt 2> gpurun_out/freplay.err || { tail -20 gpurun_out/freplay.err; exit 1; }
cut -c1-60 gpurun_out/freplay.txt; grep "add_placed\] merged\|add_placed\] resized\|filter\] host rows\|filter\] device" gpurun_out/freplay.err | tail -8
timeout -k 10 300 python -u scripts/filter_timing.py c5 c5-loose > gpurun_out/freplay2.txt 2>&1 && sed 's/ evals=.*call_ms/ call_ms/' gpurun_out/freplay2.txt | cut -c1-120
