"""The expansion call's time inside the RunOnce loop against alone: after the filter at once,
after a 2 ms pause, and a second call right after the first.  GPU box: python scripts/r6_exp_ctx.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autoscaler_amd import native, runonce  # noqa: E402
from autoscaler_amd import workloads as W  # noqa: E402

w = runonce.c5_runonce()
f = w.filt
m = native.Mirror(0)
W.load_filter(m, w.filt)
expand = runonce.DeviceExpansion()
res = {"first": [], "second": [], "after_pause": [], "c_first": [], "c_second": []}
for it in range(6):
    m.fork()
    ps = m.podset(f.pending)
    fo = m.filter_out_schedulable(f.pending, f.order, f.class_owner, f.hints, 0, podset=ps)
    unsched = f.order[fo.node < 0]
    groups = runonce._equivalence_groups(f.pending.pods, unsched)
    samples = np.array([g[0] for g in groups], np.int32)
    t = time.perf_counter()
    expand(m, ps, samples, w.templates)
    t1 = time.perf_counter()
    expand(m, ps, samples, w.templates)
    t2 = time.perf_counter()
    time.sleep(0.002)
    t3 = time.perf_counter()
    expand(m, ps, samples, w.templates)
    t4 = time.perf_counter()
    if it:
        res["first"].append((t1 - t) * 1e3)
        res["second"].append((t2 - t1) * 1e3)
        res["after_pause"].append((t4 - t3) * 1e3)
    ps.close()
    m.revert()
for k, v in res.items():
    if v:
        print(f"{k:12s} median {np.median(v):.4f} ms  all {[round(x, 4) for x in v]}")
