#!/bin/bash
# GPU-box job: bench.py with the given arguments (default: the driver's N=1 form); the JSON
# line to gpurun_out/bench_<tag>.json.  Usage: scripts/gpu_r6_bench.sh <tag> [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag="$1"; shift
timeout -k 10 900 python -u bench.py "$@" > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err; rc=$?
tail -c 3000 gpurun_out/bench_$tag.json
[[ $rc -eq 0 ]] || { echo "BENCH FAILED rc=$rc"; tail -40 gpurun_out/bench_$tag.err; exit $rc; }
