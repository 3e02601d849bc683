#!/bin/bash
# GPU-box job (round 5): estimate parity, cold C2 latency, planner phase profile, chain-wave SQ counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "estimate or plan" \
  > gpurun_out/pytest_est.log 2>&1 || { tail -30 gpurun_out/pytest_est.log; exit 1; }
tail -2 gpurun_out/pytest_est.log
timeout -k 10 120 python -u scripts/cold_est.py > gpurun_out/cold.log 2>&1 || { tail -20 gpurun_out/cold.log; exit 1; }
cat gpurun_out/cold.log
timeout -k 10 200 python -u scripts/plan_prof.py --prof > gpurun_out/plan_prof.log 2>&1 || { tail -20 gpurun_out/plan_prof.log; exit 1; }
cat gpurun_out/plan_prof.log
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
   --kernel-trace -d "$R/gpurun_out/pmc_plan1" -o run --output-format csv -- python3 "$R/scripts/plan_pmc.py" > "$R/gpurun_out/pmc_plan1.log" 2>&1 \
   || { echo PMC1 FAILED; tail -20 "$R/gpurun_out/pmc_plan1.log"; exit 1; }
cd "$R"
python3 scripts/pmc_sq.py gpurun_out/pmc_plan1 > gpurun_out/pmc_plan1.json
python3 - <<'PY'
import json
k = json.load(open("gpurun_out/pmc_plan1.json"))["kernels"]
for name, r in k.items():
    if "plan_chain" in name:
        print({x: (round(v, 3) if isinstance(v, float) else v) for x, v in r.items()})
PY
echo COLD_OK
