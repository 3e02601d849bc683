#!/bin/bash
# GPU-box job: the small legs' host/kernel split, the headline-only bench, the filter split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/r6_legs_split.py > gpurun_out/legs_split.txt 2>&1 || { tail -20 gpurun_out/legs_split.txt; exit 1; }
cat gpurun_out/legs_split.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util \
   --no-filter --no-unlimited --no-runonce --no-planner > gpurun_out/head.json 2> gpurun_out/head.err || { tail -20 gpurun_out/head.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/head.json')); print('headline ms', d['ms_per_step'], 'device', d['extra']['device_resident']['ms_per_step'], 'phases', d['extra']['phases_ms'])"
timeout -k 10 300 python -u scripts/filter_timing.py c5 c5-loose c5-loose-nohints > gpurun_out/filter_timing.txt 2>&1 || { tail -20 gpurun_out/filter_timing.txt; exit 1; }
cat gpurun_out/filter_timing.txt
