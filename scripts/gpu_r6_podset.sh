#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/r6_podset_time.py > gpurun_out/podset.txt 2>&1 || { tail -20 gpurun_out/podset.txt; exit 1; }
cat gpurun_out/podset.txt
CASIM_KNOBS=1 CASIM_DEBUG_TIMING=1 timeout -k 10 300 python -u scripts/r6_podset_time.py > gpurun_out/podset_dbg.txt 2>&1 || { tail -20 gpurun_out/podset_dbg.txt; exit 1; }
grep "^\[podset\]" gpurun_out/podset_dbg.txt | tail -6
