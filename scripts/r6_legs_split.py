"""Host/kernel split of the small C5 RunOnce legs (utilization, expansion): each native call
timed alone, median of 40 reps, on the loop's real inputs.  GPU box: python scripts/r6_legs_split.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autoscaler_amd import abi, native, runonce  # noqa: E402
from autoscaler_amd import workloads as W  # noqa: E402


def med(fn, n=40):
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts) * 1e3)


w = runonce.c5_runonce()
m = native.Mirror(0)
W.load_filter(m, w.filt)
util = runonce.DeviceUtil(0)
expand = runonce.DeviceExpansion()
m.fork()
r = runonce.run(m, util, w, expand_fn=expand)
m.revert()
print("loop ms", {k: round(v, 3) for k, v in r.ms.items()})
f = w.filt
m.fork()
fo = m.filter_out_schedulable(f.pending, f.order, f.class_owner, f.hints, 0)
ui = runonce.UtilInput(w, fo.node, "added")
print("added pods", len(ui.added_node))
out = {}
out["util_call"] = med(lambda: util(ui, w.now_ns))
t = util.table
out["set_added"] = med(lambda: t.set_added(ui.added_node, ui.added_pods))
rows = util.rows.zeros("info0", len(ui.base[0]), abi.UTIL_INFO_DTYPE, zero=False)
out["calculate_pinned"] = med(lambda: t.calculate(False, False, w.now_ns, out=rows))
out["calculate_kernel"] = t.kernel_ms
out["calculate_device_only"] = med(lambda: t.calculate(False, False, w.now_ns, to_host=False))
out["rows_zeros"] = med(lambda: util.rows.zeros("info1", len(ui.base[0]), abi.UTIL_INFO_DTYPE, zero=False))
unsched = f.order[fo.node < 0]
groups = runonce._equivalence_groups(f.pending.pods, unsched)
samples = np.array([g[0] for g in groups], np.int32)
ps = m.podset(f.pending)
out["expand_call"] = med(lambda: expand(m, ps, samples, w.templates))
out["expand_kernel"] = expand.plan.kernel_ms
pr = expand.rows.zeros("res", len(w.templates) * len(samples), abi.PRED_RESULT_DTYPE, zero=False)
out["expand_plan_run"] = med(lambda: expand.plan.run(ps, samples, out=pr.reshape(len(w.templates), len(samples))))
out["expand_tobytes"] = med(lambda: np.ascontiguousarray(w.templates).tobytes())
ps.close()
m.revert()
for k, v in out.items():
    print(f"{k:24s} {v:.4f} ms")
