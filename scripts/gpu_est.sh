#!/bin/bash
# GPU-box job: Estimate parity tests, then the headline bench alone (no legs, no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "estimate or gosort or multi or plan" > gpurun_out/pytest_est.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_est.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_est.log; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util \
   --no-filter --no-unlimited --no-runonce --no-planner > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err || { tail -20 gpurun_out/bench_head.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_head.json").read().strip().splitlines()[-1])
e = d["extra"]
print("headline", round(d["ms_per_step"], 4), "device", round(e["device_resident"]["ms_per_step"], 4),
      "i32", round(e["host_int32_ids"]["ms_per_step"], 4), "pre-chain", round(e["sort_ms"], 4), e["phases_ms"])
PY
