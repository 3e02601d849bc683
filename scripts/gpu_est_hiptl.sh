#!/bin/bash
# GPU-box job: Estimate parity tests, the headline bench alone, then a rocprofv3 HIP API +
# kernel trace of a few headline steps (host enqueue / sync timeline) into gpurun_out/hiptl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash scripts/gpu_est.sh || exit 1
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/hiptl" -o run --output-format csv -- \
   python3 "$GRAFT_REPO_ROOT/bench.py" --steps 4 --warmup 2 --no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util \
   --no-filter --no-unlimited --no-runonce --no-planner > "$GRAFT_REPO_ROOT/gpurun_out/hiptl.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/hiptl.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
find gpurun_out/hiptl -name "*.csv" | head
echo EST_HIPTL_OK
