import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
from autoscaler_amd import native, workloads as W
w = W.c3()
args_ = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
hints = np.full(len(w.table), -1, np.int32)
for limit in (20, 200):
    m = native.Mirror(0)
    W.load_sweep(m, w)
    for _ in range(6):
        m.fork()
        t = time.perf_counter()
        r = m.plan_removals(*args_, hints, 0, limit)
        dt = (time.perf_counter() - t) * 1e3
        pr = m.plan_chain_profile()
        m.revert()
        print(f"limit {limit}: {dt:.3f} ms sync {pr['sync_ms']:.3f}", flush=True)
    m.close()
