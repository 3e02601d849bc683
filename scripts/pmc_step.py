"""The C2 Estimate headline step (decoupled Go order: k_pdq_sort, k_run_table, k_emit_runs,
k_ffd_chain; results left in HBM, see PMC_MODE below) exactly STEPS times: the program the rocprofv3 --pmc passes of scripts/gpu_round.sh count
(traffic per step = total / STEPS).  PMC_LEGS=all also runs STEPS C5 FilterOutSchedulable
calls (fork/revert around each), STEPS fresh C3 sweeps and STEPS planner loops on C3 without
a limit (k_plan_chain), so their kernels are counted too."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autoscaler_amd import native, workloads as W  # noqa: E402

STEPS = int(os.environ.get("PMC_STEPS", "3"))
# PMC_MODE=device (default): the headline step with the scheduled pods left in HBM.  Under
# rocprofv3 --pmc the kernels are serialised, so the zero-copy publisher of the host-results
# mode would never see a chain start: it gives up at its start deadline and the fallback
# copies (k_narrow16, k_copy_segments) run instead — a path the timed headline never takes.
# The device-resident step runs the same sort, run table, stream and chains (less the
# chains' ticket pushes, 8 B per 4096 outputs) and k_copy_segments once at the end.
# PMC_MODE=u16 keeps the host-results call (its counters then describe the fallback).
MODE = os.environ.get("PMC_MODE", "device")
w = W.c2()
m = native.Mirror(0)
W.load_estimate(m, w)
with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
    for _ in range(STEPS):
        if MODE == "u16":
            plan.run_u16(w.max_nodes, 0, copy=False)
        else:
            plan.run(w.max_nodes, 0, copy=False, device_results=True)
m.close()
if os.environ.get("PMC_LEGS") == "all":
    import numpy as np
    f = W.c5_filter()
    g = native.Mirror(0)
    W.load_filter(g, f)
    for _ in range(STEPS):
        g.fork()
        g.filter_out_schedulable(f.pending, f.order, f.class_owner, f.hints, 0)
        g.revert()
    g.close()
    s3 = W.c3()
    m3 = native.Mirror(0)
    W.load_sweep(m3, s3)
    with native.RemovalPlan(m3, s3.candidates, s3.dest_mask, s3.cand_status, s3.move_off, s3.move_pods) as rp:
        for _ in range(STEPS):
            m3.set_hints(np.full(len(s3.table), -1, np.int32))
            rp.run(0)
    m3.close()
    m3 = native.Mirror(0)
    W.load_sweep(m3, s3)
    h0 = np.full(len(s3.table), -1, np.int32)
    for _ in range(STEPS):
        m3.fork()
        m3.plan_removals(s3.candidates, s3.dest_mask, s3.cand_status, s3.move_off, s3.move_pods, h0, 0, 0)
        m3.revert()
    m3.close()
