#!/bin/bash
# GPU-box job runner (the library is built in-tree on the CPU side beforehand).
#   scripts/gpu_job.sh tests "<pytest -k expr or file list>"   GPU tests
#   scripts/gpu_job.sh bench "<bench.py args>"                   one bench line
#   scripts/gpu_job.sh prof  "<bench.py args>"                   rocprofv3 kernel stats of a bench run
#   scripts/gpu_job.sh pmc   "<counters>|<script args>"           one rocprofv3 counter pass over a script
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
: > gpurun_out/script.log
export TMPDIR=/tmp
rc=0
while [[ $# -gt 0 ]]; do
  step="$1"; arg="$2"; shift 2
  case "$step" in
    tests)
      eval timeout -k 10 900 python -u -m pytest $arg -m gpu -x -q --timeout 300 --timeout-method thread \
        > gpurun_out/pytest_gpu.log 2>&1; rc=$?
      tail -4 gpurun_out/pytest_gpu.log
      [[ $rc -eq 0 ]] || { echo "GPU TESTS FAILED rc=$rc"; tail -60 gpurun_out/pytest_gpu.log; exit $rc; } ;;
    bench)
      timeout -k 10 600 python -u bench.py $arg > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
      [[ $rc -eq 0 ]] || { echo "BENCH FAILED rc=$rc"; tail -30 gpurun_out/bench.err; exit $rc; }
      cat gpurun_out/bench.json ;;
    prof)
      cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run \
        --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $arg > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1; rc=$?
      cd "$GRAFT_REPO_ROOT"
      [[ $rc -eq 0 ]] || { echo "PROF FAILED rc=$rc"; tail -30 gpurun_out/prof.log; exit $rc; }
      echo PROF_OK ;;
    pmc)
      ctrs="${arg%%|*}"; sargs="${arg#*|}"; tag=$(echo "$ctrs" | tr ' ' '_' | cut -c1-60)
      cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag" -o run \
        --output-format csv -- python3 $GRAFT_REPO_ROOT/$sargs > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$tag.log" 2>&1; rc=$?
      cd "$GRAFT_REPO_ROOT"
      [[ $rc -eq 0 ]] || { echo "PMC FAILED rc=$rc"; tail -30 "gpurun_out/pmc_$tag.log"; exit $rc; }
      echo "PMC_OK $tag" ;;
    script)
      echo "== $arg" >> gpurun_out/script.log
      timeout -k 10 600 python -u $arg >> gpurun_out/script.log 2>&1; rc=$?
      tail -40 gpurun_out/script.log
      [[ $rc -eq 0 ]] || { echo "SCRIPT FAILED rc=$rc"; exit $rc; } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo JOB_OK
