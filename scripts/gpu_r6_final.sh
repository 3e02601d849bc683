#!/bin/bash
# GPU-box job (round 6, closing): every GPU test, smoke, the full bench line as the driver
# runs it (N=1), the N=2 rehearsal (two ranks sharing the box's GPU over gloo), rocprofv3
# kernel statistics of the headline alone and of every leg, and the FETCH_SIZE / WRITE_SIZE
# passes (one counter per pass, --kernel-trace only) for the HBM traffic per launch.
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
timeout -k 10 600 python -u bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err \
  || { echo "BENCH N2 FAILED"; tail -20 gpurun_out/bench_n2.err; exit 1; }
tail -c 600 gpurun_out/bench_n2.json
H="--no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util --no-filter --no-unlimited --no-runonce --no-planner"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_head" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 $H > "$R/gpurun_out/prof_head.log" 2>&1 \
  || { echo "PROF HEAD FAILED"; tail -20 "$R/gpurun_out/prof_head.log"; exit 1; }
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_legs" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_legs.log" 2>&1 \
  || { echo "PROF LEGS FAILED"; tail -20 "$R/gpurun_out/prof_legs.log"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && PMC_STEPS=3 PMC_LEGS=all timeout -s KILL 180 rocprofv3 --pmc $c --kernel-trace -d "$R/gpurun_out/pmc_$c" -o run \
     --output-format csv -- python3 "$R/scripts/pmc_step.py" > "$R/gpurun_out/pmc_$c.log" 2>&1 \
     || { echo "PMC $c FAILED"; tail -20 "$R/gpurun_out/pmc_$c.log"; exit 1; }
done
cd "$R"
python3 scripts/pmc_traffic.py gpurun_out 3 > gpurun_out/pmc_traffic.json && head -c 1500 gpurun_out/pmc_traffic.json
find gpurun_out/prof_head gpurun_out/prof_legs -name "*kernel_stats.csv"
echo FINAL_OK
