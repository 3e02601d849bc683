#!/bin/bash
# GPU-box job (round 5): multi-device parity, then SQ counters of the planner chain wave alone.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py -x -q -s --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_multi.log 2>&1; rc=$?
grep -E "C3 |passed|failed|Error" gpurun_out/pytest_multi.log | tail -12
[[ $rc -eq 0 ]] || { tail -40 gpurun_out/pytest_multi.log; exit $rc; }
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
   --kernel-trace -d "$R/gpurun_out/pmc_plan1" -o run --output-format csv -- python3 "$R/scripts/plan_pmc.py" > "$R/gpurun_out/pmc_plan1.log" 2>&1 \
   || { echo PMC1 FAILED; tail -20 "$R/gpurun_out/pmc_plan1.log"; exit 1; }
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM \
   --kernel-trace -d "$R/gpurun_out/pmc_plan2" -o run --output-format csv -- python3 "$R/scripts/plan_pmc.py" > "$R/gpurun_out/pmc_plan2.log" 2>&1 \
   || { echo PMC2 FAILED; tail -20 "$R/gpurun_out/pmc_plan2.log"; exit 1; }
cd "$R"
python3 scripts/pmc_sq.py gpurun_out/pmc_plan1 > gpurun_out/pmc_plan1.json
python3 scripts/pmc_sq.py gpurun_out/pmc_plan2 > gpurun_out/pmc_plan2.json
python3 - <<'PY'
import json
for f in ("gpurun_out/pmc_plan1.json", "gpurun_out/pmc_plan2.json"):
    k = json.load(open(f))["kernels"]
    for name, r in k.items():
        if "plan_chain" in name:
            print(f, {x: (round(v, 3) if isinstance(v, float) else v) for x, v in r.items()})
PY
echo PM2_OK
