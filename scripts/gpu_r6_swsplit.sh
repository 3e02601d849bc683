#!/bin/bash
# GPU-box job: host split of the C5 RunOnce sweep call (scripts/r6_sweep_split.py), with the
# library's debug timing lines (entry to core, rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/r6_sweep_split.py > gpurun_out/swsplit.out 2> gpurun_out/swsplit.err || { tail -20 gpurun_out/swsplit.err; exit 1; }
cat gpurun_out/swsplit.out
CASIM_KNOBS=1 CASIM_DEBUG_TIMING=1 timeout -k 10 300 python -u scripts/r6_sweep_split.py > gpurun_out/swsplit_dbg.out 2> gpurun_out/swsplit_dbg.err || { tail -20 gpurun_out/swsplit_dbg.err; exit 1; }
grep "entry to core\|sync  \|\] done" gpurun_out/swsplit_dbg.err | tail -8
