"""Study (CPU, no GPU): where the planner's committing loop spends its scan work on C3, and
how much a per-64-node-block 2-D skyline of the free (cpu, memory) columns would prune.

Replays Planner.categorizeNodes (canPersist=true, planner.go:252-296) over the C3 workload
in numpy (resource-only C3: hints, rotating first fit over podDestinations minus the
candidate), checks its per-candidate eval counts against the C oracle, and reports:
  * scans (successful / failing) and the evaluations each kind costs,
  * blocks a scan reads whose per-dimension maxima pass (today's block skip) vs blocks
    whose exact skyline admits the pod (a point dominating (cpu, mem)),
  * skyline sizes per block.
Usage: python scripts/plan_skyline_study.py [n_nodes] [limit]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from autoscaler_amd import workloads as W  # noqa: E402


def skyline(c, m):
    """Pareto-maximal points of (c, m) (both larger = better)."""
    if len(c) == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    o = np.lexsort((-m, -c))              # c desc, then m desc
    cs, ms = c[o], m[o]
    keep = ms > np.maximum.accumulate(np.concatenate([[np.iinfo(np.int64).min], ms[:-1]]))
    return cs[keep], ms[keep]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    limit = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    w = W.c3(n_nodes=n)
    pods = w.table.pods
    N = len(w.nodes)
    fc = (w.nodes["alloc_milli_cpu"].astype(np.int64)).copy()
    fm = (w.nodes["alloc_memory"].astype(np.int64)).copy()
    fp = (w.nodes["alloc_pods"].astype(np.int64)).copy()
    pc = pods["req_milli_cpu"].astype(np.int64)
    pm = pods["req_memory"].astype(np.int64)
    np.subtract.at(fc, w.pod_node, pc)
    np.subtract.at(fm, w.pod_node, pm)
    np.subtract.at(fp, w.pod_node, 1)
    mask = w.dest_mask.astype(bool).copy()
    H = {}                                  # hints by pod key
    extra = [[] for _ in range(N)]
    pcpu = list(pc)
    pmem = list(pm)
    key_of = list(range(len(pc)))           # copy -> hint key of its original
    L = 0
    nb = (N + 63) // 64
    stats = {"scan_ok": 0, "scan_fail": 0, "evals_ok": 0, "evals_fail": 0, "hint": 0, "blocks_max": 0,
             "blocks_sky": 0, "blocks_fit": 0, "fail_blocks_max": 0, "fail_blocks_sky": 0, "sky_sizes": []}
    evals_per_cand = []
    removed = 0
    for ci in range(len(w.candidates)):
        if limit and removed >= limit:
            break
        node = int(w.candidates[ci])
        if w.cand_status[ci] != 0 or not mask[node]:
            evals_per_cand.append(0)
            continue
        lst = list(w.move_pods[w.move_off[ci]:w.move_off[ci + 1]]) + extra[node]
        snap = (fc.copy(), fm.copy(), fp.copy())
        for p in lst:
            fc[node] += pcpu[p]; fm[node] += pmem[p]; fp[node] += 1
        ev = 0
        dest = []
        ok_all = True
        vis = mask.copy()
        vis[node] = False
        for p in lst:
            c, m = pcpu[p], pmem[p]
            h = H.get(key_of[p], -1)
            tgt = -1
            if h >= 0:
                ev += 1
                stats["hint"] += 1
                if fc[h] >= c and fm[h] >= m and fp[h] >= 1 and h != node and mask[h]:
                    tgt = h
            if tgt < 0:
                rot = (np.arange(N) + L) % N
                v = vis[rot]
                fit = v & (fc[rot] >= c) & (fm[rot] >= m) & (fp[rot] >= 1)
                idx = np.flatnonzero(fit)
                # block-level accounting over the scanned range
                end = idx[0] if len(idx) else N - 1
                scanned = rot[: end + 1]
                blocks = np.unique(scanned // 64)
                nmax = nsky = 0
                for j in blocks:
                    lo, hi = j * 64, min(N, j * 64 + 64)
                    vv = vis[lo:hi] & (fp[lo:hi] >= 1)
                    if not vv.any():
                        continue
                    if fc[lo:hi][vv].max() >= c and fm[lo:hi][vv].max() >= m:
                        nmax += 1
                    sc, sm = skyline(fc[lo:hi][vv], fm[lo:hi][vv])
                    stats["sky_sizes"].append(len(sc))
                    if np.any((sc >= c) & (sm >= m)):
                        nsky += 1
                stats["blocks_max"] += nmax
                stats["blocks_sky"] += nsky
                e = int(v[: end + 1].sum())
                ev += e
                if len(idx):
                    # blocks between the scan's first block and the fitting one
                    d = (int(rot[idx[0]]) // 64 - int(rot[0]) // 64) % nb
                    stats.setdefault("fit_block_dist", []).append(d)
                    tgt = int(rot[idx[0]])
                    L = (L + int(idx[0]) + 1) % N
                    stats["scan_ok"] += 1
                    stats["evals_ok"] += e
                    stats["blocks_fit"] += 1
                    H[key_of[p]] = tgt
                else:
                    stats["scan_fail"] += 1
                    stats["evals_fail"] += e
                    stats["fail_blocks_max"] += nmax
                    stats["fail_blocks_sky"] += nsky
            if tgt < 0:
                ok_all = False
                break
            fc[tgt] -= c; fm[tgt] -= m; fp[tgt] -= 1
            dest.append(tgt)
        evals_per_cand.append(ev)
        if ok_all:
            for p, d in zip(lst, dest):
                pcpu.append(pcpu[p]); pmem.append(pmem[p]); key_of.append(key_of[p])
                nid = len(pcpu) - 1
                H[key_of[p]] = d
                extra[d].append(nid)
            mask[node] = False
            removed += 1
        else:
            fc[:], fm[:], fp[:] = snap
    ss = np.array(stats.pop("sky_sizes"))
    fd = np.array(stats.pop("fit_block_dist", [0]))
    print("  fitting block distance (blocks after the scan's first): " +
          "  ".join(f"{k}: {np.mean(fd == k):.3f}" for k in range(4)) + f"  >=4: {np.mean(fd >= 4):.3f}")
    print(f"C3 {N} nodes, limit {limit}: removed {removed}")
    for k, v in stats.items():
        print(f"  {k}: {v}")
    if len(ss):
        print(f"  skyline size per scanned block: mean {ss.mean():.2f}  p50 {np.median(ss):.0f}  p90 "
              f"{np.percentile(ss, 90):.0f}  p99 {np.percentile(ss, 99):.0f}  max {ss.max()}")
    if "--check" in sys.argv:
        import pyoracle
        o = pyoracle.OracleState()
        W.load_sweep(o, w)
        hints = np.full(len(w.table), -1, np.int32)
        ro = o.plan_removals(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods, hints, 0, limit)
        ev = ro.results["evals"][: len(evals_per_cand)]
        print("  evals match oracle:", bool(np.array_equal(ev, np.array(evals_per_cand))))


if __name__ == "__main__":
    main()
