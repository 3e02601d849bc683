#!/bin/bash
# GPU-box job: planner loop timings (plan_prof) twice, and the bench planner leg alone
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 200 python -u scripts/plan_prof.py 5000 > gpurun_out/plan_chk.log 2>&1 || { tail -20 gpurun_out/plan_chk.log; exit 1; }
  grep -E "^limit" gpurun_out/plan_chk.log
done
H="--no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util --no-filter --no-unlimited --no-runonce"
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 $H > gpurun_out/bench_plan.json 2> gpurun_out/bench_plan.err || { tail gpurun_out/bench_plan.err; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/bench_plan.json').read().strip().splitlines()[-1]); e = d['extra']
print({k: (round(v['gpu_ms'], 3), round(v['cpu_ms'], 3)) for k, v in e['planner']['runs'].items()})"
echo PLANCHK_OK
