"""Go 1.19 sort.Slice (pdqsort_func) — the order of Estimate's score sort
(binpacking_estimator.go:74) and FilterOutSchedulable's priority sort
(filter_out_schedulable.go:97-99).

* CPU: the C restatement (oracle/gosort.c) and the host one (autoscaler_amd/gosort.py)
  agree; the oracle's Estimate uses Go order by default.
* GPU: the device sort (csrc/pdqsort.h through ca_go_sort_ranks) returns exactly the
  restatement's permutation on every branch — insertion sort, partialInsertionSort,
  reverseRange, partitionEqual, breakPatterns, the heapSort fallback — and in every element
  store (LDS, 32-bit and 64-bit global).  Estimate's full-size parity (C2, C4) against the
  Go-order oracle is in test_gpu_parity.py.
"""
import numpy as np
import pytest

import pyoracle
from autoscaler_amd import workloads as W
from autoscaler_amd.gosort import sort_slice_desc


def test_c_and_python_restatements_agree():
    rng = np.random.default_rng(0)
    for t in range(200):
        n = int(rng.integers(0, 2500))
        keys = rng.integers(0, int(rng.integers(1, 90)), n).astype(float)
        if t % 5 == 0:
            keys = np.sort(keys)[::-1].copy()          # already sorted (partialInsertionSort path)
        elif t % 7 == 0:
            keys = np.sort(keys).copy()                # reversed (decreasingHint / reverseRange)
        pc = pyoracle.go_sort_desc(keys)
        assert sorted(pc.tolist()) == list(range(n))
        assert np.all(np.diff(keys[pc]) <= 0)
        assert pc.tolist() == sort_slice_desc(keys.tolist()), t


def test_short_slices_are_insertion_sorted():
    """n <= 12: pdqsort_func is insertionSort_func, i.e. stable."""
    rng = np.random.default_rng(1)
    for n in range(13):
        keys = rng.integers(0, 3, n).astype(float)
        assert pyoracle.go_sort_desc(keys).tolist() == np.argsort(-keys, kind="stable").tolist()


def test_break_patterns_reached():
    """C2-like inputs (64 keys, 50k pods) reach breakPatterns: the xorshift shifts (the one
    assumption not pinned by a fixture, gosort.c) decide their tie order."""
    b0, h0 = pyoracle.go_sort_stats()
    keys = np.random.default_rng(2).integers(0, 64, 50_000).astype(float)
    pyoracle.go_sort_desc(keys)
    b1, h1 = pyoracle.go_sort_stats()
    assert b1 > b0 and h1 == h0              # breakPatterns yes, heapSort fallback no


def test_limit_hook_reaches_heapsort():
    """The test hook replacing bits.Len(n) by a small limit drives pdqsort_func into its
    heapSort fallback (no natural input of this size does); the result is still a sort."""
    keys = np.random.default_rng(3).integers(0, 40, 3000).astype(float)
    _, h0 = pyoracle.go_sort_stats()
    p = pyoracle.go_sort_desc(keys, limit=2)
    _, h1 = pyoracle.go_sort_stats()
    assert h1 > h0
    assert np.all(np.diff(keys[p]) <= 0)


def _estimate(w, mode=None):
    o = pyoracle.OracleState()
    if mode is not None:
        o.set_sort_mode(mode)
    W.load_estimate(o, w)
    return o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 0)


def test_oracle_default_is_go_order():
    """The oracle's Estimate is the reference's: sort.Slice order unless told otherwise.
    On C2 the stable order schedules the same shapes slot by slot but other pods of each."""
    w = W.c2(n_pods=3000, n_groups=8, n_existing=40)
    d, g, s = _estimate(w), _estimate(w, "go"), _estimate(w, "stable")
    assert np.array_equal(d.sched_pod, g.sched_pod) and np.array_equal(d.results, g.results)
    assert np.array_equal(s.results, g.results) and s.last_index == g.last_index
    shape = lambda ids: [(int(w.table.pods[i]["req_milli_cpu"]), int(w.table.pods[i]["req_memory"])) for i in ids]
    assert shape(s.sched_pod) == shape(g.sched_pod)
    assert not np.array_equal(s.sched_pod, g.sched_pod)


def _rank_cases():
    """(ranks, limit) covering the branches of pdqsort_func at workgroup and wave sizes."""
    rng = np.random.default_rng(11)
    cases = []
    for n in (0, 1, 2, 5, 12, 13, 49, 50, 51, 200, 511, 512, 513, 700, 2000, 5000, 20000, 50368, 60000):
        for nk in (1, 2, 7, 64, 250, 4000):
            cases.append((rng.integers(0, nk, n), 0))
    for n in (600, 3000, 40000):
        k = rng.integers(0, 50, n)
        cases += [(np.sort(k), 0), (np.sort(k)[::-1].copy(), 0), (np.repeat(rng.integers(0, 60, n // 100 + 1), 100)[:n], 0)]
        s = np.sort(k)
        s[rng.integers(0, n, 4)] = rng.integers(0, 50, 4)        # nearly sorted: partialInsertionSort shifts
        cases.append((s, 0))
        cases.append((np.arange(n)[::-1] % 300, 0))              # decreasing runs: reverseRange
        cases.append((k, 2))                                      # heapSort fallback
    cases.append((rng.integers(0, 5000, 30000), 3))
    cases.append((rng.integers(0, 100000, 70000), 0))            # > 4096 ranks: 64-bit store
    return cases


@pytest.mark.gpu
@pytest.mark.parametrize("store", [0, 1, 2, 3])
def test_device_go_sort_matches_oracle(store):
    from autoscaler_amd import native
    for i, (ranks, limit) in enumerate(_rank_cases()):
        ranks = np.asarray(ranks, dtype=np.int64)
        want = pyoracle.go_sort_desc(-ranks.astype(np.float64), limit=limit)
        got = native.go_sort_ranks(ranks.astype(np.uint32), store=store, limit=limit)
        assert np.array_equal(want, got), (store, i, len(ranks), limit)


@pytest.mark.gpu
def test_device_go_sort_c2_c4_keys():
    """The exact rank sequences Estimate sorts on C2 and C4 (64 score classes, runs of 100
    identical pods per controller) for a few groups."""
    from autoscaler_amd import native
    for w in (W.c2(), W.c4(n_pods=20000, n_groups=6, n_existing=50)):
        p = w.table.pods
        for g in range(0, len(w.templates), max(1, len(w.templates) // 6)):
            idx = w.pod_idx[w.group_off[g]:w.group_off[g + 1]]
            ac = float(w.templates[g]["node"]["alloc_milli_cpu"])
            am = float(w.templates[g]["node"]["alloc_memory"])
            score = p["score_milli_cpu"][idx] / ac + p["score_memory"][idx] / am
            ranks = np.unique(-score, return_inverse=True)[1].astype(np.uint32)
            want = pyoracle.go_sort_desc(score)
            for store in (0, 2):
                assert np.array_equal(want, native.go_sort_ranks(ranks, store=store)), (w.name, g, store)


def _pis_landings(d, a, b, check):
    """Go's partialInsertionSort_func on ranks d[a:b] (less = <), recording each step's
    landing places the way the device computes them (search on the data before the swap);
    check(prev, cur) runs on consecutive steps of one call."""
    i, prev = a + 1, None
    for _ in range(5):
        while i < b and not d[i] < d[i - 1]:
            i += 1
        if i == b or b - a < 50:
            return
        ev, fv = d[i], d[i - 1]
        lo = a - 1 if a > 0 else 0
        L = i - 1
        if i - a >= 2:
            L = next((q for q in range(i - 2, lo - 1, -1) if d[q] <= ev), -1) + 1
        R = i
        if b - i >= 2:
            R = next((j for j in range(i + 1, b) if d[j] >= fv), b) - 1
        cur = (i, L, R, ev, fv)
        if prev is not None:
            check(prev, cur, a, b)
        prev = cur
        d[i], d[i - 1] = d[i - 1], d[i]
        if i - a >= 2:
            j = i - 1
            while j >= 1 and d[j] < d[j - 1]:
                d[j], d[j - 1] = d[j - 1], d[j]
                j -= 1
        if b - i >= 2:
            j = i + 1
            while j < b and d[j] < d[j - 1]:
                d[j], d[j - 1] = d[j - 1], d[j]
                j += 1


def test_pis_landing_shortcuts():
    """The device's partialInsertionSort skips a landing search when the descent repeats at
    the same i with the same moved rank (pdqsort.h PisHint): left landing = previous L + 1,
    right landing = previous R - 1.  Checked against the searches on random near-sorted
    rank sequences with repeated ranks (the C2 shape: few distinct ranks)."""
    import random
    rng = random.Random(7)
    hits = [0, 0]

    def check(prev, cur, a, b):
        pi, pL, pR, pev, pfv = prev
        i, L, R, ev, fv = cur
        if i != pi:
            return
        if i - a >= 2 and ev == pev and pL <= i - 2:
            assert L == pL + 1
            hits[0] += 1
        if b - i >= 2 and fv == pfv and pR > i:
            assert R == pR - 1
            hits[1] += 1

    for _ in range(3000):
        n = rng.randint(50, 300)
        k = rng.choice([2, 3, 5, 8, 64])
        d = sorted(rng.randrange(k) for _ in range(n))
        for _ in range(rng.randint(0, 5)):
            x, y = rng.randrange(n), rng.randrange(n)
            d[x], d[y] = d[y], d[x]
        if rng.random() < 0.5:
            cut = rng.randrange(n)
            d = d[cut:] + d[:cut]
        a = rng.randint(0, 3)
        arr = [min(d) - 1] * a + d            # a placed pivot region left of the frame
        _pis_landings(arr, a, len(arr), check)
    assert hits[0] > 100 and hits[1] > 100, hits
