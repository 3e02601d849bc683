"""Cold C2 Estimate latency (python scripts/cold_est.py): a new EstimatePlan over the full C2
batch while another plan holds its buffers (first plan: fresh device allocations), the same
after that plan is closed (buffers from the allocation cache), its first run, and the
one-shot Mirror.estimate (plan + run + teardown).  Median of 5."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autoscaler_amd import native, workloads as W  # noqa: E402

w = W.c2()
m = native.Mirror(0)
W.load_estimate(m, w)
held = native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates)
held.run_u16(w.max_nodes, 0, copy=False)
fresh, cached, first, one = [], [], [], []
for _ in range(5):
    t0 = time.perf_counter()
    p = native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates)
    fresh.append(time.perf_counter() - t0)
    p.close()
    t0 = time.perf_counter()
    with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as p:
        t1 = time.perf_counter()
        p.run_u16(w.max_nodes, 0, copy=False)
        t2 = time.perf_counter()
    cached.append(t1 - t0)
    first.append(t2 - t1)
    t0 = time.perf_counter()
    m.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 0, want_nodes=False)
    one.append(time.perf_counter() - t0)
med = lambda v: round(float(np.median(v)) * 1e3, 3)  # noqa: E731
print({"plan_create_first_ms": round(fresh[0] * 1e3, 3), "plan_create_fresh_ms": med(fresh), "plan_create_cached_ms": med(cached), "first_run_ms": med(first),
       "one_shot_estimate_ms": med(one)}, flush=True)
held.close()
m.close()
