"""Fresh C3 sweeps over D replicated mirrors (ca_multi_removal_plan; python
scripts/multi_sweep_timing.py [devices...]): wall time per run, the composition's phases
and re-runs, for D = 1, 2, 4, 8 blocks.  With one GPU every replica lives on it (the
blocks' kernels share the device: an upper bound for D GPUs); with several, block d runs
on device d % n_devices."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from autoscaler_amd import native, workloads as W  # noqa: E402

w = W.c3()
args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
nd = native.device_count() if hasattr(native, "device_count") else 1
fresh = np.full(len(w.table), -1, np.int32)
m1 = native.Mirror(0)
W.load_sweep(m1, w)
with native.RemovalPlan(m1, *args) as plan:
    ts = []
    for _ in range(8):
        m1.set_hints(fresh)
        t = time.perf_counter()
        r1 = plan.run(0)
        ts.append((time.perf_counter() - t) * 1e3)
print(f"D=1 RemovalPlan: {np.median(ts[2:]):.3f} ms", flush=True)
for D in (2, 4, 8):
    ms = []
    for d in range(D):
        m = native.Mirror(d % max(nd, 1))
        W.load_sweep(m, w)
        ms.append(m)
    with native.Multi(ms) as mm, native.MultiRemovalPlan(mm, *args) as mp:
        ts, phs = [], []
        for _ in range(8):
            t = time.perf_counter()
            g = mp.run(fresh.copy(), 0)
            ts.append((time.perf_counter() - t) * 1e3)
            phs.append(mp.stats()["phase_ms"])
        st = mp.stats()
        same = np.array_equal(g.results, r1.results) and g.last_index == r1.last_index
        ph = {k: round(float(np.median([p[k] for p in phs[2:]])), 3) for k in phs[0]}
        print(f"D={D} ca_multi: {np.median(ts[2:]):.3f} ms  phases {ph}  re-run candidates {st['rerun_candidates']}  "
              f"identical to one mirror {same}", flush=True)
    for m in ms:
        m.close()
m1.close()
