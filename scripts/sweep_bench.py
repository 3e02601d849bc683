"""C3 scale-down sweep timing: first loop (fresh hints) and the next loop (hints of the
first), HIP path vs the CPU restatement, with parity checks."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from autoscaler_amd import native, workloads as W  # noqa: E402
from pyoracle import OracleState  # noqa: E402

n_nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
w = W.c3(n_nodes=n_nodes)
g, o = native.Mirror(0), OracleState()
W.load_sweep(g, w)
W.load_sweep(o, w)
args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
for name, hints in (("fresh", np.full(len(w.table), -1, np.int32)), ("hinted", None)):
    if hints is None:
        hints = h_next
    t = time.perf_counter()
    ro = o.find_nodes_to_remove(*args, hints, 0)
    to = time.perf_counter() - t
    ts = []
    for _ in range(9):
        t = time.perf_counter()
        rg = g.find_nodes_to_remove(*args, hints, 0)
        ts.append(time.perf_counter() - t)
    ok = (np.array_equal(ro.results, rg.results) and np.array_equal(ro.dest, rg.dest)
          and np.array_equal(ro.hints, rg.hints) and ro.last_index == rg.last_index)
    tg = float(np.median(ts))
    print(f"{name}: parity={ok} oracle={to*1e3:.2f}ms gpu={tg*1e3:.3f}ms speedup={to/tg:.1f}x "
          f"removable={int(rg.results['removable'].sum())} evals={int(ro.results['evals'].sum())} "
          f"stats={g.removal_stats()}", flush=True)
    h_next = ro.hints

# inputs resident in HBM (removal plan), hints resident in the mirror
with native.RemovalPlan(g, *args) as plan:
    fresh = np.full(len(w.table), -1, np.int32)
    for name in ("plan-fresh", "plan-hinted"):
        ts = []
        for _ in range(9):
            if name == "plan-fresh":
                g.set_hints(fresh)
            t = time.perf_counter()
            r = plan.run(0)
            ts.append(time.perf_counter() - t)
        print(f"{name}: gpu={np.median(ts)*1e3:.3f}ms stats={g.removal_stats()}", flush=True)
    t = g.candidate_ticks(len(w.candidates))
    nz = t[t > 0]
    mo = np.diff(w.move_off)
    print(f"candidate us (last run): max {nz.max():.1f} p50 {np.median(nz):.1f} mean {nz.mean():.1f} n={len(nz)}; "
          f"moved pods max {mo.max()} mean {mo.mean():.1f}; slowest: {np.argsort(-t)[:5].tolist()} "
          f"{np.sort(t)[::-1][:5].round(1).tolist()} pods {mo[np.argsort(-t)[:5]].tolist()}")
