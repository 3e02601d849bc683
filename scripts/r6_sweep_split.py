"""Host split of the C5 RunOnce sweep call (FindNodesToRemove, single GPU): the loop's leg
time against the library's own total, the bare C call and the wrapper's array copies, on
the loop's real inputs at the moment the loop makes the call.  GPU box:
python scripts/r6_sweep_split.py"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from autoscaler_amd import abi, native, runonce  # noqa: E402
from autoscaler_amd import workloads as W  # noqa: E402
from autoscaler_amd.abi import ptr  # noqa: E402


def med(fn, n=15):
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts) * 1e3)


w = runonce.c5_runonce()
m = native.Mirror(0)
W.load_filter(m, w.filt)
util = runonce.DeviceUtil(0)
expand = runonce.DeviceExpansion()
orig = m.find_nodes_to_remove
out = {}


def wrapped(cand, mask, status, off, moves, hints, last_index=0):
    res = orig(cand, mask, status, off, moves, hints, last_index)
    out["C"], out["M"], out["n_hints"] = len(cand), len(moves), len(hints)
    out["wrapper"] = med(lambda: orig(cand, mask, status, off, moves, hints, last_index))
    out["lib_total"] = m.removal_stats()["total_ms"]
    c = np.ascontiguousarray(cand, np.int32)
    mk = np.ascontiguousarray(mask, np.uint8)
    stt = np.ascontiguousarray(status, np.int32)
    o = np.ascontiguousarray(off, np.int32)
    mv = np.ascontiguousarray(moves, np.int32)
    h = np.array(hints, np.int32, copy=True)
    rr = np.zeros(len(c), abi.REMOVAL_RESULT_DTYPE)
    d = np.full(max(len(mv), 1), -1, np.int32)
    li = C.c_int32(last_index)
    out["bare_c"] = med(lambda: m.lib.ca_find_nodes_to_remove(m.h, ptr(c), len(c), ptr(mk), ptr(stt), ptr(o), ptr(mv),
                                                              ptr(h), C.byref(li), ptr(rr), ptr(d)))
    out["lib_total_bare"] = m.removal_stats()["total_ms"]
    out["hints_copy"] = med(lambda: np.array(hints, np.int32, copy=True))
    return res


m.find_nodes_to_remove = wrapped
for rep in range(2):
    m.fork()
    r = runonce.run(m, util, w, expand_fn=expand)
    m.revert()
    print("loop ms", {k: round(v, 3) for k, v in r.ms.items()}, flush=True)
for k, v in out.items():
    print(f"{k:16s} {v:.4f}" if isinstance(v, float) else f"{k:16s} {v}")
