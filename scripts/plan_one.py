"""One device-chain planner call on C3 (limit from argv, default 200) for rocprofv3 passes:
scripts/gpu_job.sh pmc "<counters>|scripts/plan_one.py 200"."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autoscaler_amd import native, workloads as W  # noqa: E402

limit = int(sys.argv[1]) if len(sys.argv) > 1 else 200
w = W.c3()
m = native.Mirror(0)
W.load_sweep(m, w)
hints = np.full(len(w.table), -1, np.int32)
m.fork()
r = m.plan_removals(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods, hints, 0, limit)
m.revert()
print("ok", m.plan_stats(), int(r.results["removable"].sum()))
