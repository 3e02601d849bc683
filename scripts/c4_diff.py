"""Locate the first sched_node difference on C4 (debug)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from autoscaler_amd import native, workloads as W  # noqa: E402
import pyoracle  # noqa: E402

w = W.c4()
outs = []
for b in (pyoracle.OracleState(), native.Mirror(0)):
    W.load_estimate(b, w)
    outs.append(b.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 7))
o, g = outs
bad = np.nonzero(o.sched_node != g.sched_node)[0]
print("diffs", len(bad), "batch env", os.environ.get("CASIM_RUN_BATCH"))
if len(bad):
    i = bad[0]
    grp = int(np.searchsorted(w.group_off, i, side="right") - 1)
    a = w.group_off[grp]
    n = int(o.results[grp]["n_scheduled"])
    gb = bad[(bad >= a) & (bad < w.group_off[grp + 1])]
    print("group", grp, "first diff at", i - a, "of", n, "ndiff in group", len(gb), "results", o.results[grp])
    pods = w.table.pods
    lo, hi = max(a, i - 6), min(a + n, i + 6)
    for j in range(lo, hi):
        p = o.sched_pod[j]
        print(j - a, p, pods["req_milli_cpu"][p], pods["req_memory"][p] >> 20, "o", o.sched_node[j], "g", g.sched_node[j])
    # how many distinct groups differ
    gs = np.unique(np.searchsorted(w.group_off, bad, side="right") - 1)
    print("groups with diffs", gs[:20], len(gs))
