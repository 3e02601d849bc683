#!/bin/bash
# GPU-box job (round 5): the full bench as the driver runs it (planner leg with the
# library's per-call split), then the planner leg alone on the same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err \
  || { echo BENCH FAILED; tail -20 gpurun_out/bench_full.err; exit 1; }
python3 scripts/bench_summary.py gpurun_out/bench_full.json
python3 -c "
import json
d = json.loads(open('gpurun_out/bench_full.json').read().strip().splitlines()[-1])
print(json.dumps(d['extra']['planner']['runs'], indent=0))"
H="--no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util --no-filter --no-unlimited --no-runonce"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 $H > gpurun_out/bench_plan.json 2> gpurun_out/bench_plan.err \
  || { tail gpurun_out/bench_plan.err; exit 1; }
python3 -c "
import json
d = json.loads(open('gpurun_out/bench_plan.json').read().strip().splitlines()[-1])
print(json.dumps(d['extra']['planner']['runs'], indent=0))"
echo R5PLAN_OK
