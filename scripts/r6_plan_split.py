"""Where a planner call's time goes at limits 20 / 200 on C3 (GPU box): the Python call,
the library's own split (CASIM_DEBUG_TIMING lines on stderr) and the wrapper's marshalling.
python scripts/r6_plan_split.py"""
import os
import sys
import time

os.environ.setdefault("CASIM_KNOBS", "1")
os.environ.setdefault("CASIM_DEBUG_TIMING", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402

from autoscaler_amd import native  # noqa: E402
from autoscaler_amd import workloads as W  # noqa: E402

w = W.c3(n_nodes=5000)
args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
hints = np.full(len(w.table), -1, np.int32)
m = native.Mirror(0)
W.load_sweep(m, w)
for limit in (20, 200):
    ts = []
    for rep in range(6):
        m.fork()
        t0 = time.perf_counter()
        m.plan_removals(*args, hints, 0, limit)
        ts.append((time.perf_counter() - t0) * 1e3)
        m.revert()
        print(f"--- limit {limit} rep {rep}: {ts[-1]:.3f} ms", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    for _ in range(6):
        native.plan_args(*args, hints)
    print(f"limit {limit}: call ms median {np.median(ts[1:]):.3f} min {min(ts[1:]):.3f}; plan_args {(time.perf_counter() - t0) / 6 * 1e3:.3f} ms",
          flush=True)
