"""Host-side split of one planner call (ca_plan_removals on C3, the bench's planner leg):
the wrapper's marshalling, the C call, the library's own total, and the output wrapping,
median of 8 warm runs per limit (scripts/gpu_r5_ab.sh)."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autoscaler_amd import native, workloads as W  # noqa: E402
from autoscaler_amd.native import plan_args, ptr, _check  # noqa: E402

w = W.c3(n_nodes=5000)
args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
hints = np.full(len(w.table), -1, np.int32)
for limit in (20, 200, 0):
    m = native.Mirror(0)
    W.load_sweep(m, w)
    rows = []
    for rep in range(9):
        m.fork()
        t0 = time.perf_counter()
        a = plan_args(*args, hints)
        t1 = time.perf_counter()
        li = C.c_int32(0)
        nm = C.c_int32(0)
        _check(m.lib.ca_plan_removals(m.h, ptr(a.cand), len(a.cand), ptr(a.mask), ptr(a.status), ptr(a.off),
                                      ptr(a.moves), int(limit), a.pdb_ptr, ptr(a.hints), len(a.hints),
                                      C.byref(li), ptr(a.res), ptr(a.out_moves), len(a.out_moves), C.byref(nm)),
               "ca_plan_removals")
        t2 = time.perf_counter()
        out = a.output(li.value, nm.value)
        t3 = time.perf_counter()
        del a, out
        t4 = time.perf_counter()
        st = m.plan_stats()
        m.revert()
        rows.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3, st["total_ms"], (t3 - t2) * 1e3, (t4 - t3) * 1e3))
    r = np.median(np.array(rows[1:]), axis=0)
    print(f"limit {limit}: plan_args {r[0]:.3f}  C call {r[1]:.3f} (library total {r[2]:.3f})  output {r[3]:.3f}  "
          f"free {r[4]:.3f} ms", flush=True)
    m.close()
