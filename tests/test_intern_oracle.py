"""Interning + the oracle's bitset filter chain vs the API-level restatement.

For random clusters (taints, selectors, affinity terms incl. parse errors, host
ports, extended resources, unschedulable nodes...) every (pending pod, node)
CheckPredicates verdict and every FitsAnyNode answer of the oracle must equal the
string-level evaluation in tests/apifilters.py.
"""
import pytest

from apifilters import filters, prefilter
from autoscaler_amd.clustersnapshot import ClusterSnapshot
from autoscaler_amd.predicatechecker import SchedulerBasedPredicateChecker
from randgen import rand_cluster


def _snapshot(backend, nodes, scheduled):
    snap = ClusterSnapshot(backend)
    snap.AddNodes(nodes)
    for p, n in scheduled:
        snap.AddPod(p, n)
    return snap


@pytest.mark.parametrize("seed", range(12))
def test_check_predicates_matches_api_filters(seed, oracle_lib):
    rng, nodes, scheduled, pending = rand_cluster(seed)
    snap = _snapshot(oracle_lib.OracleState(), nodes, scheduled)
    snap.ensure(pods=pending)
    pc = SchedulerBasedPredicateChecker()
    on_node = {n.name: [p for p, m in scheduled if m == n.name] for n in nodes}
    for pod in pending:
        for node in nodes:
            err = pc.CheckPredicates(snap, pod, node.name)
            if prefilter(pod) == "fail":
                assert err is not None and err.ErrorType() == 1
                continue
            want = filters(pod, node, on_node[node.name])
            got = None if err is None else err.PredicateName()
            assert got == want, f"seed {seed} pod {pod.name} node {node.name}: oracle {got} api {want}"


@pytest.mark.parametrize("seed", range(12))
def test_fits_any_node_matches_api_scan(seed, oracle_lib):
    rng, nodes, scheduled, pending = rand_cluster(seed)
    snap = _snapshot(oracle_lib.OracleState(), nodes, scheduled)
    snap.ensure(pods=pending)
    pc = SchedulerBasedPredicateChecker()
    on_node = {n.name: [p for p, m in scheduled if m == n.name] for n in nodes}
    last = 0
    for pod in pending:
        pc.last_index = last
        name, err = pc.FitsAnyNode(snap, pod)
        # reference loop (schedulerbased.go:114-134) over API objects
        pf = prefilter(pod)
        want = None
        if pf != "fail":
            for i in range(len(nodes)):
                node = nodes[(last + i) % len(nodes)]
                if pf is not None and node.name not in pf:
                    continue
                if node.unschedulable:
                    continue
                if filters(pod, node, on_node[node.name], apply_unsched=False) is None:
                    want = node.name
                    last = (last + i + 1) % len(nodes)
                    break
        assert (None if err else name) == want, f"seed {seed} pod {pod.name}"
        assert pc.last_index == last
