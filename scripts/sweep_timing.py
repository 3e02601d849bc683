"""C3 sweep timing through the removal plan (python scripts/sweep_timing.py [n_nodes]):
fresh and hinted loops, wall time per call, the library's own timings, CPU port time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

from autoscaler_amd import native  # noqa: E402
from autoscaler_amd import workloads as W  # noqa: E402
import pyoracle  # noqa: E402

n_nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
w = W.c3(n_nodes=n_nodes)
m = native.Mirror(0)
W.load_sweep(m, w)
args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
fresh = np.full(len(w.table), -1, np.int32)
with native.RemovalPlan(m, *args) as plan:
    for mode in ("fresh", "hinted"):
        ts, st = [], []
        for _ in range(12):
            if mode == "fresh":
                m.set_hints(fresh)
            t = time.perf_counter()
            r = plan.run(0)
            ts.append((time.perf_counter() - t) * 1e3)
            st.append(m.removal_stats())
        print(mode, "call_ms median", round(float(np.median(ts)), 3), "min", round(min(ts), 3),
              "lib total", round(float(np.median([s["total_ms"] for s in st])), 3),
              "kernel", round(float(np.median([s["kernel_ms"] for s in st])), 3),
              "rounds", st[-1]["rounds"], flush=True)
o = pyoracle.OracleState()
W.load_sweep(o, w)
t = time.perf_counter()
o.find_nodes_to_remove(*args, fresh, 0)
print("cpu fresh ms", round((time.perf_counter() - t) * 1e3, 3))

# per-candidate device time of the last exact pass (ticks of 10 ns) and moved-pod counts
with native.RemovalPlan(m, *args) as plan:
    m.set_hints(fresh)
    plan.run(0)
    us = m.candidate_ticks(len(w.candidates))
    pods = np.diff(w.move_off)
    ran = us > 0
    print("exact-pass candidates", int(ran.sum()), "us p50/p90/p99/max",
          [round(float(np.percentile(us[ran], q)), 1) for q in (50, 90, 99, 100)])
    top = np.argsort(-us)[:8]
    print("slowest:", [(int(c), round(float(us[c]), 1), int(pods[c])) for c in top])
    print("us per moved pod p50", round(float(np.median(us[ran] / np.maximum(pods[ran], 1))), 2))

# where the wrapper's time goes: the bare C call vs RemovalPlan.run
import ctypes as C  # noqa: E402
from autoscaler_amd.abi import ptr  # noqa: E402
with native.RemovalPlan(m, *args) as plan:
    res = np.zeros(len(w.candidates), plan.results.dtype)
    bare, full = [], []
    for _ in range(12):
        li = C.c_int32(0)
        t = time.perf_counter()
        m.lib.ca_removal_plan_run(plan.h, None, C.byref(li), ptr(res), None)
        bare.append((time.perf_counter() - t) * 1e3)
        t = time.perf_counter()
        plan.run(0)
        full.append((time.perf_counter() - t) * 1e3)
    print("hinted: bare C call ms", round(float(np.median(bare)), 3), "RemovalPlan.run ms",
          round(float(np.median(full)), 3), "lib total", round(m.removal_stats()["total_ms"], 3))
