"""The C2 Estimate step, device-resident results, exactly STEPS times: the program the
rocprofv3 --pmc passes of scripts/gpu_round.sh count (traffic per step = total / STEPS)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autoscaler_amd import native, workloads as W  # noqa: E402

STEPS = int(os.environ.get("PMC_STEPS", "3"))
w = W.c2()
m = native.Mirror(0)
W.load_estimate(m, w)
with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
    for _ in range(STEPS):
        plan.run(w.max_nodes, 0, copy=False, device_results=True)
m.close()
