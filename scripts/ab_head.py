"""A/B of a run-time switch on the bench's headline step (C2, results on the host as 16-bit
podset indices through the zero-copy publisher, phase events off), interleaved in one
process.  Usage: python scripts/ab_head.py VAR [rounds]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["CASIM_KNOBS"] = "1"            # (read once, before the library loads)
from autoscaler_amd import native, workloads as W  # noqa: E402

var = sys.argv[1]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 12
w = W.c2()
m = native.Mirror(0)
W.load_estimate(m, w)
res = {"off": [], "on": []}
with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
    plan.set_phase_timing(False)
    for r in range(rounds):
        for mode in ("off", "on"):
            if mode == "on":
                os.environ[var] = "1"
            else:
                os.environ.pop(var, None)
            for _ in range(3):
                plan.run_u16(w.max_nodes, 0, copy=False)
            t = time.perf_counter()
            for _ in range(30):
                plan.run_u16(w.max_nodes, 0, copy=False)
            res[mode].append((time.perf_counter() - t) / 30 * 1e3)
for k, v in res.items():
    print(f"{var}={'1' if k == 'on' else 'unset'}: median {np.median(v):.4f} ms  min {np.min(v):.4f}  max {np.max(v):.4f}")
