#!/bin/bash
# GPU-box job: chain section cycles (CASIM_PROF build), and the CW=2 chain variant's headline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
CASIM_LIB_PATH=$PWD/autoscaler_amd/lib/libcasim_prof.so timeout -k 10 200 python -u scripts/chain_diag.py > gpurun_out/chain_diag.log 2>&1 || { tail gpurun_out/chain_diag.log; exit 1; }
cat gpurun_out/chain_diag.log
H="--no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util --no-filter --no-unlimited --no-runonce --no-planner"
CASIM_LIB_PATH=$PWD/autoscaler_amd/lib/cw2/libcasim.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 $H > gpurun_out/ab_cw2.json 2>gpurun_out/ab_cw2.err || { tail gpurun_out/ab_cw2.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/ab_cw2.json").read().strip().splitlines()[-1])
e = d["extra"]
print("cw2 headline", round(d["ms_per_step"], 4), "chain", round(e["phases_ms"]["chain_ms"], 4), "device", round(e["device_resident"]["ms_per_step"], 4))
PY
