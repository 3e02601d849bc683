#!/bin/bash
# GPU-box job: which earlier bench leg slows the planner leg's first (limit 20) mirror
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
ALL="--no-sweep --no-c4 --no-unlimited --no-expansion --no-util --no-filter --no-runonce"
for keep in runonce filter sweep; do
  F=$(echo $ALL | sed "s/--no-$keep//")
  timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline $F > gpurun_out/bench_bis.json 2> gpurun_out/bench_bis.err || { tail gpurun_out/bench_bis.err; exit 1; }
  python3 -c "
import json
d = json.loads(open('gpurun_out/bench_bis.json').read().strip().splitlines()[-1]); e = d['extra']
print('$keep', {k: round(v['gpu_ms'], 3) for k, v in e['planner']['runs'].items()})"
done
echo BISECT_OK
