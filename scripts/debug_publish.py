"""Compare published (zero-copy) Estimate results with the device-copy path on C2."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autoscaler_amd import native, workloads as W  # noqa: E402

w = W.c2()
m = native.Mirror(0)
W.load_estimate(m, w)
with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
    ref = plan.run(w.max_nodes, 0, want_nodes=True)           # device copy path
    for it in range(2):
        p = plan.run(w.max_nodes, 0, want_nodes=False)        # publishing path
        bad = np.nonzero(ref.sched_pod != p.sched_pod)[0]
        print("iter", it, "mismatches", len(bad))
        off = w.group_off
        for i in bad[:10]:
            g = int(np.searchsorted(off, i, side="right") - 1)
            j = i - off[g]
            print(f"  idx {i} group {g} out {j} chunk {j // 4096} n_sched {int(ref.results[g]['n_scheduled'])}"
                  f" count {off[g+1]-off[g]} ref {ref.sched_pod[i]} got {p.sched_pod[i]}")
        gs = sorted(set(int(np.searchsorted(off, i, side='right') - 1) for i in bad))
        print("  groups", gs[:20], len(gs))
