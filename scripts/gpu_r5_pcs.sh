#!/bin/bash
# GPU-box job (round 5): host-trap PC sampling of the planner chain wave (no limit, helpers off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
   --pc-sampling-interval 1 -d "$R/gpurun_out/pcs" -o run --output-format csv -- python3 "$R/scripts/plan_pmc.py" \
   > "$R/gpurun_out/pcs.log" 2>&1 || { echo PCS FAILED; tail -30 "$R/gpurun_out/pcs.log"; exit 1; }
ls -la "$R/gpurun_out/pcs" "$R"/gpurun_out/pcs/* | head -20
tail -5 "$R/gpurun_out/pcs.log"
echo PCS_OK
