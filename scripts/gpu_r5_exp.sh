#!/bin/bash
# GPU-box job (round 5): expansion plan tests, RunOnce parity, and the bench's expansion + RunOnce legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_scaleup.py tests/test_runonce.py -x -q -m gpu --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_exp.log 2>&1 || { tail -40 gpurun_out/pytest_exp.log; exit 1; }
tail -2 gpurun_out/pytest_exp.log
timeout -k 10 400 python -u bench.py --steps 5 --no-sweep --no-c4 --no-util --no-filter --no-unlimited --no-planner \
  > gpurun_out/bench_exp.json 2> gpurun_out/bench_exp.err || { tail -30 gpurun_out/bench_exp.err; exit 1; }
python3 - <<'PY'
import json
r = json.loads(open("gpurun_out/bench_exp.json").read().strip().splitlines()[-1])
e = r["extra"]
print("headline", r["ms_per_step"])
for k, v in e["expansion"].items():
    if isinstance(v, dict):
        print(k, {x: (round(y, 4) if isinstance(y, float) else y) for x, y in v.items()})
ro = e["c5_runonce"]
print("runonce gpu", {k: round(v, 3) for k, v in ro["gpu_ms"].items()})
print("runonce cpu", {k: round(v, 3) for k, v in ro.get("cpu_ms", {}).items()})
print("speedup", {k: round(v, 2) for k, v in ro.get("speedup", {}).items()}, ro.get("parity"))
PY
echo EXP_OK
