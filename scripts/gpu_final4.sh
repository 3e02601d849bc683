#!/bin/bash
# Round-4 measurement job: the full bench line, rocprofv3 kernel stats of the headline and of
# the legs, the planner's phase profile.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "decoupled or cross_class" > gpurun_out/pytest_f4.log 2>&1 || { tail -40 gpurun_out/pytest_f4.log; exit 1; }
tail -2 gpurun_out/pytest_f4.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python3 scripts/bench_summary.py gpurun_out/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run \
   --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-sweep --no-c4 \
   --no-expansion --no-util --no-filter --no-unlimited --no-runonce --no-planner \
   > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo PROF FAILED; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_legs" -o run \
   --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline \
   > "$GRAFT_REPO_ROOT/gpurun_out/prof_legs.log" 2>&1 || { echo PROF LEGS FAILED; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_legs.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u scripts/plan_prof.py 5000 --prof > gpurun_out/plan_prof.log 2>&1 || { tail -20 gpurun_out/plan_prof.log; exit 1; }
cat gpurun_out/plan_prof.log
timeout -k 10 200 python -u scripts/pdq_prof.py > gpurun_out/pdq_prof.log 2>&1 || { tail -20 gpurun_out/pdq_prof.log; exit 1; }
cat gpurun_out/pdq_prof.log
echo FINAL4_OK
