"""A/B timing of a run-time switch (an environment variable read by the library on every
run) on the C2 (or C4) Estimate step, device-resident results, interleaved in one process.
Usage: python scripts/ab_env.py VAR [c2|c4] [rounds]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the library reads its switches only when CASIM_KNOBS (or CASIM_TEST_HOOKS) was set when it
# first checked (once per process, casim_internal.h knobs_enabled): set it before loading
os.environ["CASIM_KNOBS"] = "1"
from autoscaler_amd import native, workloads as W  # noqa: E402

var = sys.argv[1]
wl = sys.argv[2] if len(sys.argv) > 2 else "c2"
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 10
w = W.c2() if wl == "c2" else W.c4()
m = native.Mirror(0)
W.load_estimate(m, w)
res = {"off": [], "on": []}
with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
    for r in range(rounds):
        for mode in ("off", "on"):
            if mode == "on":
                os.environ[var] = "1"
            else:
                os.environ.pop(var, None)
            plan.run(w.max_nodes, 0, copy=False, device_results=True)
            t = time.perf_counter()
            for _ in range(20):
                plan.run(w.max_nodes, 0, copy=False, device_results=True)
            res[mode].append((time.perf_counter() - t) / 20 * 1e3)
for k, v in res.items():
    print(f"{var}={'1' if k == 'on' else 'unset'}: median {np.median(v):.4f} ms  min {np.min(v):.4f}  max {np.max(v):.4f}")
