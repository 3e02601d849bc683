"""Per-group chain diagnostics on the C2 batch: device time per group and single-pod steps."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autoscaler_amd import native, workloads as W  # noqa: E402

w = W.c2()
m = native.Mirror(0)
W.load_estimate(m, w)
plan = native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates)
for _ in range(3):
    out = plan.run(w.max_nodes, 0, want_nodes=False, copy=False)   # the bench configuration
d = plan.group_ticks()
r = out.results
order = np.argsort(-d[:, 0])
print("phases", plan.stats()["phases"])
print("chain us: max %.1f mean %.1f median %.1f" % (d[:, 0].max(), d[:, 0].mean(), np.median(d[:, 0])))
for g in order[:12]:
    t = w.templates[g]["node"]
    print(f"g{g:3d} {d[g,0]:8.1f}us single={int(d[g,1])} nodes={int(r[g]['nodes_added'])} sched={int(r[g]['n_scheduled'])}"
          f" evals={int(r[g]['evals'])} cpu={int(t['alloc_milli_cpu'])} mem={int(t['alloc_memory'])>>30}Gi")

if os.environ.get("CASIM_LIB_PATH", "").endswith("libcasim_prof.so"):
    import ctypes as C
    lib = native.load()
    G = len(w.templates)
    buf = np.zeros((G, 15), np.uint64)
    lib.ca_debug_chain_prof(buf.ctypes.data_as(C.POINTER(C.c_uint64)), G)
    names = ["run_end", "capa", "revol", "update", "open", "total", "n_rev", "n_runs", "prologue", "post_bar", "exhausted", "run_total", "loop_top", "epilogue", "pre_loop"]
    for g in order[:6]:
        print(f"g{g:3d} " + " ".join(f"{n}={int(v)}" for n, v in zip(names, buf[g])))

    if hasattr(lib, "ca_debug_rt_prof"):
        rt = np.zeros((G, 4), np.uint64)
        plan.run_u16(w.max_nodes, 0, copy=False)
        lib.ca_debug_rt_prof(rt.ctypes.data_as(C.POINTER(C.c_uint64)), G)
        print("k_run_table cycles (ranking, counting, scan, records), heaviest groups:")
        for g in order[:6]:
            print(f"g{g:3d} " + " ".join(str(int(v)) for v in rt[g]))
