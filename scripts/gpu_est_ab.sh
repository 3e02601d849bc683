#!/bin/bash
# GPU-box job: Estimate parity tests, then the headline alone three times (box spread)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "estimate or gosort or multi or plan or publisher" > gpurun_out/pytest_est.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_est.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_est.log; exit $rc; }
H="--no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util --no-filter --no-unlimited --no-runonce --no-planner"
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 40 --warmup 3 $H > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err || { tail gpurun_out/bench_head.err; exit 1; }
  python3 -c "
import json
d = json.loads(open('gpurun_out/bench_head.json').read().strip().splitlines()[-1]); e = d['extra']
print('headline', round(d['ms_per_step'], 4), 'device', round(e['device_resident']['ms_per_step'], 4), 'i32', round(e['host_int32_ids']['ms_per_step'], 4))"
done
CASIM_LIB_PATH=$PWD/autoscaler_amd/lib/libcasim_prof.so timeout -k 10 200 python -u scripts/chain_diag.py > gpurun_out/chain_diag.log 2>&1 || { tail gpurun_out/chain_diag.log; exit 1; }
grep -A8 "k_run_table cycles" gpurun_out/chain_diag.log
echo EST_AB_OK
