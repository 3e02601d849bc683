#!/bin/bash
# GPU-box job: selected GPU tests, then the full default bench (N=1).
# Usage: scripts/gpu_r6_job.sh <tag> <pytest args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag="$1"; shift
if [[ $# -gt 0 ]]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > gpurun_out/pytest_$tag.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_$tag.log
  [[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; tail -60 gpurun_out/pytest_$tag.log; exit $rc; }
fi
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err; rc=$?
[[ $rc -eq 0 ]] || { echo "BENCH FAILED rc=$rc"; tail -40 gpurun_out/bench_$tag.err; exit $rc; }
python scripts/r6_summary.py gpurun_out/bench_$tag.json
