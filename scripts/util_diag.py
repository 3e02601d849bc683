"""Timing of the RunOnce utilization step's parts on the device (set_added, calculate)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autoscaler_amd import native, runonce  # noqa: E402

w = runonce.c5_runonce()
placed = np.full(len(w.filt.order), -1, np.int32)
rng = np.random.default_rng(0)
sel = rng.random(len(placed)) < 0.85
placed[sel] = rng.integers(0, len(w.filt.nodes), int(sel.sum()))
ui = runonce.UtilInput(w, placed, "added")
t = native.UtilTable(0, *ui.base)
rows = native.PinnedRows()
out = rows.zeros("info", len(w.filt.nodes), native.abi.UTIL_INFO_DTYPE)
du = runonce.DeviceUtil(0)
for rep in range(5):
    t0 = time.perf_counter()
    t.set_added(ui.added_node, ui.added_pods)
    t1 = time.perf_counter()
    r = t.calculate(False, False, w.now_ns)
    t2 = time.perf_counter()
    r2 = t.calculate(False, False, w.now_ns, to_host=False)
    t3 = time.perf_counter()
    t.set_added(ui.added_node, ui.added_pods)
    t4 = time.perf_counter()
    r3 = t.calculate(False, False, w.now_ns, out=out)
    t5 = time.perf_counter()
    r4 = du(ui, w.now_ns)
    t6 = time.perf_counter()
    assert np.array_equal(r.view(np.uint8), r3.view(np.uint8)) and np.array_equal(r.view(np.uint8), r4.view(np.uint8))
    print(f"set_added {1e3*(t1-t0):.3f} ms  calculate(to host) {1e3*(t2-t1):.3f} ms  calculate(device) {1e3*(t3-t2):.3f} ms  "
          f"calculate(page-locked, zero-copy) {1e3*(t5-t4):.3f} ms  DeviceUtil {1e3*(t6-t5):.3f} ms  kernel {t.kernel_ms:.4f} ms", flush=True)
