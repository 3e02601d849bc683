"""FilterOutSchedulable on the CPU restatement.

The batched entry point (or_filter_out_schedulable: the whole TrySchedulePods loop of
filter_out_schedulable.go:95-124 in one call, similar-pods cache and hints included) must
give exactly what the facade's pod-by-pod HintingSimulator.TrySchedulePods gives over the
same backend (hinting_simulator.go:58-125, similar_pods.go:43-111): statuses, lastIndex,
evaluations, overflowing controllers and hints.  Pinned by the reference's own table
(tests/golden: filter_out_schedulable/*).
"""
import numpy as np
import pytest

from autoscaler_amd import workloads as W
from autoscaler_amd.clustersnapshot import ClusterSnapshot
from autoscaler_amd.podlistprocessor import FilterOutSchedulablePodListProcessor, PodPriority, TrySchedulePodsAnywhere
from autoscaler_amd.predicatechecker import SchedulerBasedPredicateChecker
from autoscaler_amd.simulator import HintingSimulator, SimilarPodsScheduling
from fosgen import rand_filter_case


def _snapshot(backend, nodes, scheduled):
    s = ClusterSnapshot(backend)
    s.AddNodes(nodes)
    for p, n in scheduled:
        s.AddPod(p, n)
    return s


def run_both(make_backend, seed, n_nodes=10, n_pending=60, last_index=0):
    """(sequential facade result, batched result) on fresh snapshots of one case."""
    nodes, scheduled, pending, hints = rand_filter_case(seed, n_nodes, n_pending)
    pending.sort(key=lambda p: -PodPriority(p))
    out = []
    for batched in (False, True):
        snap = _snapshot(make_backend(), nodes, scheduled)
        pc = SchedulerBasedPredicateChecker()
        pc.last_index = last_index
        sim = HintingSimulator(pc)
        sim.hints.current = dict(hints)
        if batched:
            st, ov = TrySchedulePodsAnywhere(sim, snap, list(pending))
        else:
            st, ov, _ = sim.TrySchedulePods(snap, list(pending), None, False)
        out.append({"statuses": [(s.pod.name, s.node_name) for s in st], "overflow": ov, "L": pc.last_index,
                    "evals": pc.evals, "hints": dict(sim.hints.current),
                    "pods": sorted((p.name, n.node.name) for n in snap.List() for p in n.pods)})
    return out


@pytest.mark.parametrize("seed", range(16))
def test_batched_equals_sequential_oracle(seed, oracle_lib):
    seq, bat = run_both(oracle_lib.OracleState, seed, last_index=seed % 7)
    assert bat == seq


def test_similar_pods_cap_overflows(oracle_lib):
    """A controller with 12 failing variants: 10 are remembered, the 11th overflows."""
    from autoscaler_amd import k8s
    nodes = [k8s.build_test_node("n0", 1000, 1 << 30)]
    pending = []
    for v in range(12):
        for j in range(3):
            p = k8s.build_test_pod(f"v{v}-{j}", 2000 + v, 1)
            p.owner_refs = [k8s.OwnerReference("ReplicaSet", "rs", "rs")]
            pending.append(p)
    res = []
    for batched in (False, True):
        snap = _snapshot(oracle_lib.OracleState(), nodes, [])
        pc = SchedulerBasedPredicateChecker()
        sim = HintingSimulator(pc)
        if batched:
            st, ov = TrySchedulePodsAnywhere(sim, snap, list(pending))
        else:
            st, ov, _ = sim.TrySchedulePods(snap, list(pending), None, False)
        res.append((len(st), ov, pc.evals))
    # 10 remembered variants scan once each; variants 10 and 11 scan for every pod
    assert res[0] == res[1] == (0, 1, 10 + 2 * 3)
    assert SimilarPodsScheduling.max_pods_per_owner_ref == 10


def test_processor_priority_order_and_hint_generations(oracle_lib):
    nodes, scheduled, pending, hints = rand_filter_case(3, 8, 40)
    snap = _snapshot(oracle_lib.OracleState(), nodes, scheduled)
    proc = FilterOutSchedulablePodListProcessor(SchedulerBasedPredicateChecker())
    proc.schedulingSimulator.hints.current = dict(hints)
    cand = list(pending)
    still = proc.filterOutSchedulableByPacking(cand, snap)
    prios = [PodPriority(p) for p in cand]
    assert prios == sorted(prios, reverse=True)                       # :97-99
    assert [p.name for p in still] == [p.name for p in cand if p.name in {q.name for q in still}]
    # DropOldHints (:121): this call's hints became the old generation
    h = proc.schedulingSimulator.hints
    assert h.current == {} and len(h.old) >= len(cand) - len(still)


@pytest.mark.parametrize("taints", [False, True])
def test_c5_filter_oracle_idempotent(taints, oracle_lib):
    """Size-independent property: the pods still pending after a call stay pending in a
    second call on the resulting state (placements only take capacity away; a similar-pods
    skip copies the failure of an identical pod)."""
    w = W.c5_filter(n_nodes=1500, pods_per_node=20, n_pending=4000, taints=taints)
    o = oracle_lib.OracleState()
    W.load_filter(o, w)
    r = o.filter_out_schedulable(w.pending, w.order, w.class_owner, w.hints, 0)
    assert 0 < r.placed < len(w.order)
    left = w.order[r.node < 0]
    r2 = o.filter_out_schedulable(w.pending, left, w.class_owner, None, r.last_index)
    assert r2.placed == 0 and r2.last_index == r.last_index
    assert np.array_equal(r.hints[r.node >= 0], r.node[r.node >= 0])
