"""Go 1.19 sort.Slice restatements (oracle/gosort.c, autoscaler_amd/gosort.py) and the
tie-order gap between the reference's pdqsort and the device's stable order.

sort.Slice is Estimate's score sort (binpacking_estimator.go:74) and FilterOutSchedulable's
priority sort (filter_out_schedulable.go:97-99).  Ties come out in pdqsort order, so:
  * C2 (ties only between resource-identical pods): counts, lastIndex and every placement
    decision are the same in both orders; only WHICH of the identical pods fills a slot
    differs (the scheduled-pod identities);
  * C4-style ties (same shape, different tolerations / selectors): the orders can place
    different pods, so the device (stable) result is exact against the stable restatement
    only — the gap these tests measure.
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


def _estimate(w, mode):
    o = pyoracle.OracleState()
    o.set_sort_mode(mode)
    W.load_estimate(o, w)
    return o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 0)


def test_c2_ties_only_change_pod_identity():
    w = W.c2(n_pods=3000, n_groups=8, n_existing=40)
    s, g = _estimate(w, "stable"), _estimate(w, "go")
    assert np.array_equal(s.results, g.results) and s.last_index == g.last_index
    assert np.array_equal(s.sched_node, g.sched_node)
    shape = lambda ids: [(int(w.table.pods[i]["req_milli_cpu"]), int(w.table.pods[i]["req_memory"])) for i in ids]
    assert shape(s.sched_pod) == shape(g.sched_pod)          # the same shapes, slot by slot
    assert not np.array_equal(s.sched_pod, g.sched_pod)      # ... but other pods of each shape


def test_c4_tie_gap_measured():
    """C4 ties are between pods that differ in tolerations / selectors: the two orders can
    schedule different pods; the device is pinned to the stable restatement (H2)."""
    w = W.c4(n_pods=5000, n_groups=12, n_existing=100)
    s, g = _estimate(w, "stable"), _estimate(w, "go")
    order_diff = int((s.sched_pod != g.sched_pod).sum())
    assert order_diff > 0
    sets_diff = sum(set(s.sched_pod[a:b].tolist()) != set(g.sched_pod[a:b].tolist())
                    for a, b in zip(w.group_off[:-1], w.group_off[1:]))
    print(f"C4 tie gap: {order_diff} output slots, {sets_diff} groups with different pod sets, "
          f"count changes {int((s.results['node_count'] != g.results['node_count']).sum())}")
