"""Per-step diagnostics of the C5 RunOnce loop on the GPU (python scripts/runonce_diag.py):
the sweep's and the filter's internal statistics at C5 scale."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

from autoscaler_amd import native, runonce  # noqa: E402
from autoscaler_amd import workloads as W  # noqa: E402

if "--phases" in sys.argv:
    os.environ["CASIM_DEBUG_TIMING"] = "1"
    os.environ["CASIM_KNOBS"] = "1"
w = runonce.c5_runonce()
m = native.Mirror(0)
W.load_filter(m, w.filt)




util = runonce.DeviceUtil(0)
expand = runonce.DeviceExpansion()


for rep in range(3):
    m.fork()
    r = runonce.run(m, util, w, expand_fn=expand)
    print({k: round(v, 2) for k, v in r.ms.items()}, flush=True)
    print("filter", m.filter_stats(), flush=True)
    print("sweep", m.removal_stats(), flush=True)
    m.revert()
