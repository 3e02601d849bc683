#!/bin/bash
# GPU-box job: build, GPU tests, smoke, bench, rocprof kernel stats.  Every GPU step has
# its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP="${1:-all}"
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail gpurun_out/build.log; exit 1; }
if [[ "$STEP" == all || "$STEP" == tests ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -5 gpurun_out/pytest_gpu.log
  [[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
fi
if [[ "$STEP" == all || "$STEP" == smoke ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
if [[ "$STEP" == all || "$STEP" == bench ]]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [[ "$STEP" == all || "$STEP" == prof ]]; then
  # the headline alone (the bench line's kernel averages come from these launches only),
  # then the other legs in a profile of their own
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run \
     --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-sweep --no-c4 \
     --no-expansion --no-util --no-filter --no-unlimited --no-runonce --no-planner \
     > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo PROF FAILED; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_legs" -o run \
     --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline \
     > "$GRAFT_REPO_ROOT/gpurun_out/prof_legs.log" 2>&1 || { echo PROF LEGS FAILED; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_legs.log"; exit 1; }
  cd "$GRAFT_REPO_ROOT"
  echo PROF_OK
fi
if [[ "$STEP" == pmc ]]; then
  # HBM traffic: one counter per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950)
  for c in FETCH_SIZE WRITE_SIZE; do
    cd /tmp && PMC_STEPS=3 timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c" -o run \
       --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/pmc_step.py" \
       > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c.log" 2>&1 || { echo "PMC $c FAILED"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c.log"; exit 1; }
  done
  cd "$GRAFT_REPO_ROOT"
  python3 scripts/pmc_traffic.py gpurun_out 3 > gpurun_out/pmc_traffic.json && cat gpurun_out/pmc_traffic.json
fi
echo ROUND_OK
