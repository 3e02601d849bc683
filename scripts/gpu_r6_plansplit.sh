#!/bin/bash
# GPU-box job: the planner call's split at limits 20 / 200 (scripts/r6_plan_split.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/r6_plan_split.py > gpurun_out/plansplit.out 2> gpurun_out/plansplit.err || { tail -20 gpurun_out/plansplit.err; exit 1; }
cat gpurun_out/plansplit.out
grep "plan chain\|^---\|\[planner\]" gpurun_out/plansplit.err | tail -40
