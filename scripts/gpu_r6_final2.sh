#!/bin/bash
# GPU-box job (round 6, after the chain / publisher changes): every GPU test, smoke, the N=1
# bench line as the driver runs it, and the headline's rocprofv3 kernel statistics.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu2.log 2>&1 \
  || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/pytest_gpu2.log; exit 1; }
tail -1 gpurun_out/pytest_gpu2.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke2.log; exit 1; }
tail -1 gpurun_out/smoke2.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench2.json 2> gpurun_out/bench2.err \
  || { echo BENCH FAILED; tail -20 gpurun_out/bench2.err; exit 1; }
python3 scripts/bench_summary.py gpurun_out/bench2.json
H="--no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util --no-filter --no-unlimited --no-runonce --no-planner"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_head2" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 $H > "$R/gpurun_out/prof_head2.log" 2>&1 \
  || { echo "PROF HEAD FAILED"; tail -20 "$R/gpurun_out/prof_head2.log"; exit 1; }
cd "$R"
f=$(find gpurun_out/prof_head2 -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_timeline.py "$f" > gpurun_out/tl2.txt && python3 scripts/rocprof_chain_span.py "$f" 2>/dev/null | tail -3
echo FINAL2_OK
