"""ScaleUp option computation (§8f "next" #2): BuildPodGroups, the (node group x pod
group) feasibility matrix of ComputeExpansionOption, and the options' Estimate batch.

CPU: the grouping rules of equivalence/groups.go:59-112, and the oracle's matrix
(fork, add the template copy, CheckPredicates, revert — orchestrator.go:455-482)
against the API-level filter restatement (tests/apifilters.py).  GPU: the device
matrix (ca_check_templates) and the whole option computation bit-exact vs the oracle.
"""
import copy
import random

import numpy as np
import pytest

from apifilters import filters, prefilter
from autoscaler_amd import abi
from autoscaler_amd.clustersnapshot import ClusterSnapshot, NodeInfo
from autoscaler_amd.estimator import ThresholdBasedEstimationLimiter
from autoscaler_amd.k8s import OwnerReference, build_test_pod
from autoscaler_amd.predicatechecker import SchedulerBasedPredicateChecker
from autoscaler_amd.scaleup import BuildPodGroups, ComputeExpansionOptions
from estgen import _encode_estimate, _estimate_inputs


def _owned(name, uid, cpu=100, mem=1 << 20, kind="ReplicaSet", labels=None):
    p = build_test_pod(name, cpu, mem)
    p.owner_refs = [OwnerReference(kind, uid, uid)]
    if labels:
        p.labels = dict(labels)
    return p


def test_build_pod_groups_rules():
    a = [_owned(f"a{i}", "rs-a") for i in range(3)]                        # one group
    b = [_owned("b0", "rs-a", cpu=200)]                                     # same owner, other spec
    c = [_owned("c0", "rs-a", labels={"x": "1"})]                           # same owner, other labels
    d = [_owned(f"d{i}", "ds-1", kind="DaemonSet") for i in range(2)]      # DaemonSet pods: alone
    e = [build_test_pod("e0", 100, 1 << 20), build_test_pod("e1", 100, 1 << 20)]   # no controller: alone
    pods = [a[0], b[0], a[1], c[0], d[0], e[0], a[2], d[1], e[1]]
    groups = BuildPodGroups(pods)
    names = [[p.name for p in g.pods] for g in groups]
    assert names == [["a0", "a1", "a2"], ["b0"], ["c0"], ["d0"], ["e0"], ["d1"], ["e1"]]


def test_build_pod_groups_overflow_per_controller():
    # groups.go:57,79-86: at most 10 remembered groups per controller; later distinct
    # pods of that controller each get a fresh group that is never matched again
    pods = [_owned(f"p{i}", "rs", cpu=100 + i) for i in range(12)] + [_owned("q", "rs", cpu=100 + 11)]
    groups = BuildPodGroups(pods)
    assert len(groups) == 13
    assert [len(g.pods) for g in groups] == [1] * 13


@pytest.mark.parametrize("seed", range(10))
def test_oracle_template_matrix_matches_api_filters(seed, oracle_lib):
    rng, nodes, pods, templates, groups = _estimate_inputs(seed, n_groups=8, n_pods=60)
    table, node_recs, tm, off, pod_idx = _encode_estimate(nodes, pods, templates, groups)
    o = oracle_lib.OracleState()
    if len(node_recs):
        o.add_nodes(node_recs)
    res = o.check_templates(table, np.arange(len(pods), dtype=np.int32), tm)
    for g, (t, ds) in enumerate(templates):
        for e, pod in enumerate(pods):
            r = res[g, e]
            if prefilter(pod) == "fail":
                assert int(r["type"]) == abi.CA_PRED_INTERNAL
                continue
            want = filters(pod, t, ds)
            got = None if int(r["type"]) == abi.CA_PRED_OK else abi.PLUGIN_NAMES[int(r["plugin"])]
            assert got == want, (seed, g, pod.name, got, want)
    assert o.node_count() == len(node_recs)          # every fork reverted


def _snapshot_for(backend, nodes):
    snap = ClusterSnapshot(backend)
    snap.AddNodes(nodes)
    return snap


def _options_inputs(seed):
    rng, nodes, pods, templates, _ = _estimate_inputs(seed, n_groups=10, n_pods=90)
    # controllers so that pod groups have several members
    for i, p in enumerate(pods):
        if rng.random() < 0.7:
            p.owner_refs = [OwnerReference("ReplicaSet", f"rs{i % 5}", f"rs{i % 5}")]
    extra = []
    for p in pods[:30]:
        if p.owner_refs:
            q = copy.deepcopy(p)
            q.name = p.name + "-twin"
            extra.append(q)
    pods = pods + extra
    random.Random(seed).shuffle(pods)
    infos = [(f"ng{g}", NodeInfo(t, list(ds))) for g, (t, ds) in enumerate(templates)]
    return nodes, pods, infos


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_check_templates_gpu_matches_oracle(seed, oracle_lib):
    from autoscaler_amd import native
    rng, nodes, pods, templates, groups = _estimate_inputs(seed, n_groups=12, n_pods=150)
    table, node_recs, tm, off, pod_idx = _encode_estimate(nodes, pods, templates, groups)
    samples = np.arange(len(pods), dtype=np.int32)
    outs = []
    for b in (oracle_lib.OracleState(), native.Mirror(0)):
        if len(node_recs):
            b.add_nodes(node_recs)
        outs.append(b.check_templates(table, samples, tm))
    assert np.array_equal(outs[0], outs[1])
    v = b.check_templates(table, samples, tm, verdict_only=True)          # the one-byte verdicts
    assert np.array_equal(v.astype(bool), outs[0]["type"] == abi.CA_PRED_OK)
    # the resident plan (ca_expansion_plan): pageable and page-locked outputs, two runs
    ps = b.podset(table)
    with native.ExpansionPlan(b, tm) as plan:
        assert np.array_equal(plan.run(ps, samples), outs[0])
        assert np.array_equal(plan.run(ps, samples, verdict_only=True), v)
        pin = native.PinnedRows()
        out = pin.zeros("r", len(tm) * len(samples), abi.PRED_RESULT_DTYPE).reshape(len(tm), len(samples))
        assert np.array_equal(plan.run(ps, samples[::-1].copy(), out=out), outs[0][:, ::-1])
        pin.close()
        assert plan.run(ps, samples[:0]).shape == (len(tm), 0)
        with pytest.raises(native.CasimError):
            plan.run(ps, np.array([len(pods)], np.int32))                  # outside the pod set
    ps.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_compute_expansion_options_gpu_matches_oracle(seed, oracle_lib):
    from autoscaler_amd import native
    res = []
    for backend in (oracle_lib.OracleState(), native.Mirror(0)):
        nodes, pods, infos = _options_inputs(seed)
        snap = _snapshot_for(backend, nodes)
        pc = SchedulerBasedPredicateChecker()
        pc.last_index = seed % 3
        groups = BuildPodGroups(pods)
        opts, feas = ComputeExpansionOptions(snap, pc, groups, infos, ThresholdBasedEstimationLimiter(max_nodes=7))
        res.append(([(o.node_group, o.node_count, [p.name for p in o.pods]) for o in opts],
                    [(g.schedulable, sorted((k, int(v["plugin"]), int(v["reasons"])) for k, v in
                                            g.scheduling_errors.items())) for g in groups],
                    feas, pc.last_index, pc.evals))
    (oo, og, of, ol, oe), (go, gg, gf, gl, ge) = res
    assert oo == go
    assert og == gg
    assert np.array_equal(of, gf)
    assert ol == gl and oe == ge


@pytest.mark.gpu
def test_check_templates_full_c4(oracle_lib):
    """The bench's expansion leg at full size: every C4 pod (50k) against 100 templates."""
    from autoscaler_amd import native
    from autoscaler_amd import workloads as W
    w = W.c4()
    samples = np.arange(len(w.table.pods), dtype=np.int32)
    outs = []
    for b in (oracle_lib.OracleState(), native.Mirror(0)):
        W.load_estimate(b, w)
        outs.append(b.check_templates(w.table, samples, w.templates))
    assert np.array_equal(outs[0], outs[1])
    assert 0 < int((outs[1]["type"] == 0).sum()) < outs[1].size
