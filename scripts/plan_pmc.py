"""The planner loop on C3 (no limit) once after a warm-up run, for rocprofv3 --pmc passes of
k_plan_chain (python scripts/plan_pmc.py [limit]).  CASIM_PLAN_HELPERS=0 (set here unless
given) runs the chain wave alone, so the SQ counters describe it and not the helpers."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["CASIM_KNOBS"] = "1"
os.environ.setdefault("CASIM_PLAN_HELPERS", "0")
import numpy as np  # noqa: E402
from autoscaler_amd import native, workloads as W  # noqa: E402

limit = int(sys.argv[1]) if len(sys.argv) > 1 else 0
w = W.c3()
m = native.Mirror(0)
W.load_sweep(m, w)
h = np.full(len(w.table), -1, np.int32)
for _ in range(2):
    m.fork()
    m.plan_removals(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods, h, 0, limit)
    print(m.plan_chain_profile()["kernel_ms"], flush=True)
    m.revert()
m.close()
