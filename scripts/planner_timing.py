"""Planner (canPersist=true) loop on C3: device time, speculation rounds and conflicts,
the oracle's time, parity.  Usage: python scripts/planner_timing.py [n_nodes ...]"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

from autoscaler_amd import native  # noqa: E402
from autoscaler_amd import workloads as W  # noqa: E402
import pyoracle  # noqa: E402


def run(n_nodes: int, limit: int, reps: int = 3) -> None:
    w = W.c3(n_nodes=n_nodes)
    args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
    hints = np.full(len(w.table), -1, np.int32)
    o = pyoracle.OracleState()
    W.load_sweep(o, w)
    t0 = time.perf_counter()
    po = o.plan_removals(*args, hints, 0, limit)
    t_cpu = time.perf_counter() - t0
    m = native.Mirror(0)
    W.load_sweep(m, w)
    best, first = 1e9, None
    for _ in range(reps):                      # the first run also uploads the snapshot
        m.fork()
        t0 = time.perf_counter()
        pm = m.plan_removals(*args, hints, 0, limit)
        best = min(best, time.perf_counter() - t0)
        st = m.plan_stats()
        m.revert()
        first = first or pm                    # (later runs number their copies after the detached ones)
    pm = first
    ok = (np.array_equal(po.results, pm.results) and np.array_equal(po.moves, pm.moves)
          and np.array_equal(po.hints, pm.hints) and po.last_index == pm.last_index)
    rem = int(po.results["removable"].sum())
    ran = int((po.results["reason"] != 101).sum())
    print(f"C3 n={n_nodes} limit={limit}: removable {rem}, candidates run {ran}, gpu {best * 1e3:.2f} ms "
          f"(rounds {st['rounds']}, conflicts {st['conflicts']}, simulated {st['simulated']}), "
          f"cpu port {t_cpu * 1e3:.2f} ms, parity {ok}", flush=True)
    m.close()


if __name__ == "__main__":
    sizes = [int(a) for a in sys.argv[1:]] or [5000]
    for n in sizes:
        for lim in (20, 200, 0):
            run(n, lim)
