#!/bin/bash
# GPU-box job: the expansion call in the RunOnce context (scripts/r6_exp_ctx.py), plain and
# with the library's host split (CASIM_DEBUG_TIMING).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/r6_exp_ctx.py > gpurun_out/expctx.txt 2>&1 || { tail -20 gpurun_out/expctx.txt; exit 1; }
cat gpurun_out/expctx.txt
CASIM_KNOBS=1 CASIM_DEBUG_TIMING=1 timeout -k 10 300 python -u scripts/r6_exp_ctx.py > gpurun_out/expctx_dbg.txt 2> gpurun_out/expctx_dbg.err || { tail -20 gpurun_out/expctx_dbg.err; exit 1; }
cat gpurun_out/expctx_dbg.txt
grep "\[expansion\]" gpurun_out/expctx_dbg.err | tail -9
