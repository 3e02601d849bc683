#!/bin/bash
# GPU-box job: Estimate GPU tests, then the headline alone (results on the host).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_c_abi.py -m gpu -x -q --timeout 120 --timeout-method thread -k "estimate or abi" > gpurun_out/pytest_est.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_est.log
[ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_est.log; exit $rc; }
H="--no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util --no-filter --no-unlimited --no-runonce --no-planner"
for r in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 $H > gpurun_out/b_head.json 2>gpurun_out/b_head.err || { tail gpurun_out/b_head.err; exit 1; }
python scripts/bench_summary.py gpurun_out/b_head.json | head -2
python -c "import json;d=json.loads(open('gpurun_out/b_head.json').read().strip().splitlines()[-1]);print({k:round(v,4) for k,v in d['extra']['phases_ms'].items()})"
done
