#!/bin/bash
# GPU-box job: Estimate headline with chain workgroups of 4 / 8 / 16 waves (A/B builds in
# autoscaler_amd/lib/cwN), full-C2 parity for each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
H="--no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util --no-filter --no-unlimited --no-runonce --no-planner"
for v in cw1; do
  if [ $v = base ]; then L=$PWD/autoscaler_amd/lib/libcasim.so; else L=$PWD/autoscaler_amd/lib/$v/libcasim.so; fi
  CASIM_LIB_PATH=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 $H > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || { tail gpurun_out/ab_$v.err; exit 1; }
  python - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
e = d["extra"]
print(sys.argv[1], "headline", round(d["ms_per_step"], 4), "chain", round(e["phases_ms"]["chain_ms"], 4),
      "device", round(e["device_resident"]["ms_per_step"], 4), flush=True)
PY
  CASIM_LIB_PATH=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "estimate" > gpurun_out/ab_$v.pytest 2>&1 || { tail -20 gpurun_out/ab_$v.pytest; exit 1; }
  tail -1 gpurun_out/ab_$v.pytest
done
