#!/bin/bash
# GPU-box job: the C5 RunOnce sweep's host-walk misses (CASIM_DEBUG_TIMING): which rows miss
# against the last re-centring pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/runonce_diag.py --phases > gpurun_out/rdiag.out 2> gpurun_out/rdiag.err || { tail -20 gpurun_out/rdiag.err; exit 1; }
cat gpurun_out/rdiag.out
grep "miss at\|table round\|\] done" gpurun_out/rdiag.err | tail -30
