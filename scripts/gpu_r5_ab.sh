#!/bin/bash
# GPU-box job (round 5): A/B of a library variant (autoscaler_amd/lib/alt, altp = its prof build)
# against the default one on the planner: parity of the variant, then release timings and the
# phase profile of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ALT=autoscaler_amd/lib/alt/libcasim.so
ALTP=autoscaler_amd/lib/altp/libcasim_prof.so
CASIM_LIB_PATH=$ALT timeout -k 10 300 python -u -m pytest tests/test_gpu_planner.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_planner_alt.log 2>&1 || { tail -30 gpurun_out/pytest_planner_alt.log; exit 1; }
tail -2 gpurun_out/pytest_planner_alt.log
for v in base alt base alt; do
  if [[ $v == alt ]]; then export CASIM_LIB_PATH=$ALT; else unset CASIM_LIB_PATH; fi
  timeout -k 10 200 python -u scripts/plan_prof.py > gpurun_out/plan_rel_$v.log 2>&1 || { tail -20 gpurun_out/plan_rel_$v.log; exit 1; }
  echo "== $v"; grep -E "^limit|host:" gpurun_out/plan_rel_$v.log
done
unset CASIM_LIB_PATH
timeout -k 10 200 python -u scripts/plan_prof.py --prof > gpurun_out/plan_prof_base.log 2>&1 || { tail -20 gpurun_out/plan_prof_base.log; exit 1; }
CASIM_LIB_PATH=$ALTP timeout -k 10 200 python -u scripts/plan_prof.py > gpurun_out/plan_prof_alt.log 2>&1 || { tail -20 gpurun_out/plan_prof_alt.log; exit 1; }
echo "== prof base"; cat gpurun_out/plan_prof_base.log
echo "== prof alt"; cat gpurun_out/plan_prof_alt.log
CASIM_DEBUG_TIMING=1 timeout -k 10 200 python -u scripts/plan_prof.py > gpurun_out/plan_dbg.log 2>&1 || { tail -20 gpurun_out/plan_dbg.log; exit 1; }
echo "== debug timing"; grep -E "^limit|plan chain|plan_args" gpurun_out/plan_dbg.log
echo AB_OK
