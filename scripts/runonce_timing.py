"""C5 RunOnce legs on the GPU, a few loops (python scripts/runonce_timing.py): the legs'
times per loop; with CASIM_DEBUG_TIMING=1 the library's own phase marks go to stderr."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autoscaler_amd import native, runonce  # noqa: E402
from autoscaler_amd import workloads as W  # noqa: E402

w = runonce.c5_runonce()
m = native.Mirror(0)
W.load_filter(m, w.filt)
util = runonce.DeviceUtil(0)
expand = runonce.DeviceExpansion()
for i in range(4):
    m.fork()
    print(f"[loop {i}] start", file=sys.stderr, flush=True)
    r = runonce.run(m, util, w, expand_fn=expand)
    m.revert()
    print(i, {k: round(v, 3) for k, v in r.ms.items()}, flush=True)
expand.close()
util.close()
m.close()
