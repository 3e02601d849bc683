#!/bin/bash
# GPU-box job: rocprofv3 kernel trace of the headline steps alone; timeline into gpurun_out/tl.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/tl" -o run --output-format csv -- \
   python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util \
   --no-filter --no-unlimited --no-runonce --no-planner > "$GRAFT_REPO_ROOT/gpurun_out/tl.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/tl.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
f=$(find gpurun_out/tl -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_timeline.py "$f" > gpurun_out/tl.txt
wc -l gpurun_out/tl.txt
