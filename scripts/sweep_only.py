"""Run the C3 sweep a few times on cuda:0 (for counter collection)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autoscaler_amd import native, workloads as W  # noqa: E402

w = W.c3(n_nodes=int(sys.argv[1]) if len(sys.argv) > 1 else 5000)
g = native.Mirror(0)
W.load_sweep(g, w)
hints = np.full(len(w.table), -1, np.int32)
for _ in range(3):
    r = g.find_nodes_to_remove(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods, hints, 0)
print("removable", int(r.results["removable"].sum()), g.removal_stats())
