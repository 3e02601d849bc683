#!/bin/bash
# Round-4 closing measurement job: every GPU test, the full bench line, rocprofv3 kernel
# stats of the headline and of the legs, PMC traffic passes, the sort's per-step profile.
# Each GPU step has its own limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log
[[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python3 scripts/bench_summary.py gpurun_out/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run \
   --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-sweep --no-c4 \
   --no-expansion --no-util --no-filter --no-unlimited --no-runonce --no-planner \
   > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo PROF FAILED; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_legs" -o run \
   --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline \
   > "$GRAFT_REPO_ROOT/gpurun_out/prof_legs.log" 2>&1 || { echo PROF LEGS FAILED; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_legs.log"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && PMC_STEPS=3 PMC_LEGS=all timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c" -o run \
     --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/pmc_step.py" \
     > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c.log" 2>&1 || { echo "PMC $c FAILED"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c.log"; exit 1; }
done
cd "$GRAFT_REPO_ROOT"
python3 scripts/pmc_traffic.py gpurun_out 3 > gpurun_out/pmc_traffic.json && echo PMC_OK
timeout -k 10 200 python -u scripts/pdq_prof.py > gpurun_out/pdq_prof.log 2>&1 || { tail -20 gpurun_out/pdq_prof.log; exit 1; }
echo FINAL5_OK
