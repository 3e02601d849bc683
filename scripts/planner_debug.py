"""One planner run on C3 (limit 0) for CASIM_DEBUG_TIMING traces: per planner round the
build / speculation / validation split, per sweep the table rounds and kernel times.
Usage: CASIM_DEBUG_TIMING=1 python scripts/planner_debug.py [n_nodes] [limit]"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

from autoscaler_amd import native  # noqa: E402
from autoscaler_amd import workloads as W  # noqa: E402

n_nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
limit = int(sys.argv[2]) if len(sys.argv) > 2 else 0
w = W.c3(n_nodes=n_nodes)
hints = np.full(len(w.table), -1, np.int32)
m = native.Mirror(0)
W.load_sweep(m, w)
m.fork()
t0 = time.perf_counter()
pm = m.plan_removals(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods, hints, 0, limit)
dt = time.perf_counter() - t0
print(f"plan: {dt * 1e3:.2f} ms, stats {m.plan_stats()}", flush=True)
m.revert()
m.close()
