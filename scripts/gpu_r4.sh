#!/bin/bash
# Round-4 GPU-box job: GPU tests, planner phase profile (CASIM_PROF build), PMC traffic
# passes of the round-4 kernels.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP="${1:-all}"
if [[ "$STEP" == all || "$STEP" == tests ]]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_gpu.log
  [[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
fi
if [[ "$STEP" == all || "$STEP" == planprof ]]; then
  timeout -k 10 200 python -u scripts/plan_prof.py 5000 --prof > gpurun_out/plan_prof.log 2>&1 || { echo PLANPROF FAILED; tail -20 gpurun_out/plan_prof.log; exit 1; }
  cat gpurun_out/plan_prof.log
fi
if [[ "$STEP" == all || "$STEP" == bench ]]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
  python3 scripts/bench_summary.py gpurun_out/bench.json 2>/dev/null || head -c 3000 gpurun_out/bench.json
fi
if [[ "$STEP" == all || "$STEP" == filter ]]; then
  timeout -k 10 300 python -u scripts/filter_timing.py --phases c5-loose-nohints c5-loose c5 > gpurun_out/filter_timing.log 2>&1 || { echo FILTER TIMING FAILED; tail -20 gpurun_out/filter_timing.log; exit 1; }
  grep -v "^\[" gpurun_out/filter_timing.log | tail -5
fi
if [[ "$STEP" == all || "$STEP" == multi ]]; then
  # N = 2 rehearsal of the weak-scaling path on the one GPU (two ranks share it; gloo collectives)
  CASIM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
     --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 \
     > gpurun_out/multi2.json 2> gpurun_out/multi2.err || { echo MULTI FAILED; tail -20 gpurun_out/multi2.err; exit 1; }
  tail -c 1500 gpurun_out/multi2.json
fi
if [[ "$STEP" == all || "$STEP" == pmc ]]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    cd /tmp && PMC_STEPS=3 PMC_LEGS=all timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c" -o run \
       --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/pmc_step.py" \
       > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c.log" 2>&1 || { echo "PMC $c FAILED"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc_$c.log"; exit 1; }
  done
  cd "$GRAFT_REPO_ROOT"
  python3 scripts/pmc_traffic.py gpurun_out 3 > gpurun_out/pmc_traffic.json && echo PMC_OK
fi
echo JOB_OK
