"""Podset creation time at C5 (the RunOnce filter leg uploads the pending pods first):
python scripts/r6_podset_time.py (GPU box)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autoscaler_amd import native, runonce  # noqa: E402
from autoscaler_amd import workloads as W  # noqa: E402

w = runonce.c5_runonce()
m = native.Mirror(0)
W.load_filter(m, w.filt)
ts = []
for _ in range(8):
    t = time.perf_counter()
    ps = m.podset(w.filt.pending)
    ts.append((time.perf_counter() - t) * 1e3)
    ps.close()
f = w.filt
ps = m.podset(f.pending)
tf = []
for _ in range(4):
    m.fork()
    t = time.perf_counter()
    m.filter_out_schedulable(f.pending, f.order, f.class_owner, f.hints, 0, podset=ps)
    tf.append((time.perf_counter() - t) * 1e3)
    m.revert()
print(f"podset create ms median {np.median(ts[1:]):.3f} min {min(ts[1:]):.3f} ({len(f.pending.pods)} pods); "
      f"filter with podset ms median {np.median(tf[1:]):.3f}")
