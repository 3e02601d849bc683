"""Developer check: HIP path vs oracle on C1/C2/C3 (scaled), with timings."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from autoscaler_amd import native, workloads as W  # noqa: E402
from pyoracle import OracleState  # noqa: E402


def cmp_est(name, w):
    o = OracleState()
    g = native.Mirror(0)
    W.load_estimate(o, w)
    W.load_estimate(g, w)
    t = time.time()
    ro = o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 0)
    to = time.time() - t
    with native.EstimatePlan(g, w.table, w.group_off, w.pod_idx, w.templates) as plan:
        rg = plan.run(w.max_nodes, 0)
        t = time.time()
        rg = plan.run(w.max_nodes, 0)
        tg = time.time() - t
        st = plan.stats()
    ok = (np.array_equal(ro.results, rg.results) and np.array_equal(ro.sched_pod, rg.sched_pod)
          and np.array_equal(ro.sched_node, rg.sched_node) and ro.last_index == rg.last_index)
    if not ok:
        print(" results eq", np.array_equal(ro.results, rg.results), "sp eq", np.array_equal(ro.sched_pod, rg.sched_pod),
              "sn eq", np.array_equal(ro.sched_node, rg.sched_node), "L", ro.last_index, rg.last_index)
    ev = int(ro.results["evals"].sum())
    print(f"{name}: parity={ok} oracle={to*1e3:.1f}ms gpu={tg*1e3:.2f}ms stats={st} evals={ev} "
          f"L={ro.last_index}/{rg.last_index}", flush=True)
    if not ok:
        bad = np.nonzero(ro.results != rg.results)[0][:5]
        print(" oracle", ro.results[bad])
        print(" gpu   ", rg.results[bad])
        pods = w.table.pods
        for g in range(len(w.templates)):
            a, b = w.group_off[g], w.group_off[g + 1]
            n = ro.results[g]["n_scheduled"]
            so, sg = ro.sched_pod[a:a + n], rg.sched_pod[a:a + n]
            no, ng = ro.sched_node[a:a + n], rg.sched_node[a:a + n]
            if np.array_equal(so, sg) and np.array_equal(no, ng):
                continue
            d = int(np.nonzero((so != sg) | (no != ng))[0][0])
            t = w.templates[g]["node"]
            def score(pi):
                p = pods[pi]
                return p["score_milli_cpu"] / t["alloc_milli_cpu"] + p["score_memory"] / t["alloc_memory"]
            print(f" group {g} first diff at {d}/{n}: oracle pod {so[d]} node {no[d]} score {score(so[d])!r} | "
                  f"gpu pod {sg[d]} node {ng[d]} score {score(sg[d])!r}; prev oracle {so[max(d-3,0):d+3]} "
                  f"gpu {sg[max(d-3,0):d+3]} nodes o {no[max(d-3,0):d+3]} g {ng[max(d-3,0):d+3]}")
            break
    return ok


def cmp_sweep(name, w):
    o = OracleState()
    g = native.Mirror(0)
    W.load_sweep(o, w)
    W.load_sweep(g, w)
    hints = np.full(len(w.table), -1, np.int32)
    t = time.time()
    ro = o.find_nodes_to_remove(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods, hints, 0)
    to = time.time() - t
    rg = g.find_nodes_to_remove(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods, hints, 0)
    ts = []
    for _ in range(7):
        t = time.time()
        rg = g.find_nodes_to_remove(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods, hints, 0)
        ts.append(time.time() - t)
    tg = float(np.median(ts))
    ok = (np.array_equal(ro.results, rg.results) and np.array_equal(ro.dest, rg.dest)
          and np.array_equal(ro.hints, rg.hints) and ro.last_index == rg.last_index)
    print(f"{name}: parity={ok} oracle={to*1e3:.1f}ms gpu={tg*1e3:.2f}ms stats={g.removal_stats()} "
          f"evals={int(ro.results['evals'].sum())} L={ro.last_index}/{rg.last_index}", flush=True)
    if not ok:
        bad = np.nonzero(ro.results != rg.results)[0][:5]
        print(" oracle", ro.results[bad])
        print(" gpu   ", rg.results[bad])
    return ok


if __name__ == "__main__":
    which = sys.argv[1:] or ["c1", "c2s", "c3s", "c2", "c3"]
    allok = True
    if "c1" in which:
        allok &= cmp_est("C1", W.c1())
    if "c2s" in which:
        allok &= cmp_est("C2-small", W.c2(n_pods=5000, n_groups=10, n_existing=100))
    if "c3s" in which:
        allok &= cmp_sweep("C3-small", W.c3(n_nodes=500))
    if "c3" in which:
        allok &= cmp_sweep("C3", W.c3())
    if "c2" in which:
        allok &= cmp_est("C2", W.c2())
    print("ALL_OK" if allok else "MISMATCH")
