#!/bin/bash
# GPU-box job (round 5, closing): every GPU test, smoke, the full bench line as the driver
# runs it, and rocprofv3 kernel statistics of the headline alone and of every leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
  || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err \
  || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python3 scripts/bench_summary.py gpurun_out/bench.json
H="--no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util --no-filter --no-unlimited --no-runonce --no-planner"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_head" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 $H > "$R/gpurun_out/prof_head.log" 2>&1 \
  || { echo "PROF HEAD FAILED"; tail -20 "$R/gpurun_out/prof_head.log"; exit 1; }
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_legs" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_legs.log" 2>&1 \
  || { echo "PROF LEGS FAILED"; tail -20 "$R/gpurun_out/prof_legs.log"; exit 1; }
cd "$R"
find gpurun_out/prof_head gpurun_out/prof_legs -name "*kernel_stats.csv" | head
echo FINAL_OK
