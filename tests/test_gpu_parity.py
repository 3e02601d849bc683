"""HIP path (libcasim.so through the C ABI) vs the CPU restatement: bit-exact.

Parity is exact equality of every output: node counts, scheduled pods and their
node ordinals, removable sets, destinations, hints, lastIndex and the number of
filter evaluations.  Sizes are chosen so the oracle finishes in seconds; the
full-size workloads are also checked through size-independent properties.
"""
import random

import numpy as np
import pytest

from autoscaler_amd import abi, native
from autoscaler_amd import workloads as W
from autoscaler_amd.clustersnapshot import ClusterSnapshot, NodeInfo
from autoscaler_amd.intern import Interner
from autoscaler_amd.predicatechecker import SchedulerBasedPredicateChecker
from golden_runner import load_cases, run_case
from randgen import rand_cluster, rand_node, rand_pod
from estgen import _encode_estimate, _estimate_inputs

pytestmark = pytest.mark.gpu

CASES = load_cases()


@pytest.fixture(scope="module")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle


def _mirror():
    return native.Mirror(0)


# --------------------------------------------------------------------------
# the reference's own known-answer tests
# --------------------------------------------------------------------------
@pytest.mark.parametrize("case", CASES, ids=[c["id"] for c in CASES])
def test_reference_case_on_gpu(case):
    errs = run_case(case, _mirror)
    assert not errs, f"{case['source']}: {errs}"


# --------------------------------------------------------------------------
# predicate checker: random clusters
# --------------------------------------------------------------------------
def _both(oracle, nodes, scheduled):
    snaps = []
    for b in (oracle.OracleState(), _mirror()):
        s = ClusterSnapshot(b)
        s.AddNodes(nodes)
        for p, n in scheduled:
            s.AddPod(p, n)
        snaps.append(s)
    return snaps


@pytest.mark.parametrize("seed", range(8))
def test_check_predicates_random(seed, oracle):
    rng, nodes, scheduled, pending = rand_cluster(seed, n_nodes=10, n_pods=30)
    so, sg = _both(oracle, nodes, scheduled)
    table_o = so.encode(pending)
    table_g = sg.encode(pending)
    for i in range(len(pending)):
        for pos in range(len(nodes)):
            assert so.backend.check_predicates(table_o, i, pos) == sg.backend.check_predicates(table_g, i, pos), \
                (seed, i, pos)
    # dense feasibility matrix == CheckPredicates verdicts
    mat = sg.backend.fits_matrix(table_g)
    for i in range(len(pending)):
        for pos in range(len(nodes)):
            t = so.backend.check_predicates(table_o, i, pos)[0]
            assert mat[i, pos] == (1 if t == abi.CA_PRED_OK else 0)


@pytest.mark.parametrize("seed", range(8))
def test_fits_any_node_random(seed, oracle):
    rng, nodes, scheduled, pending = rand_cluster(seed, n_nodes=12, n_pods=40)
    so, sg = _both(oracle, nodes, scheduled)
    to, tg = so.encode(pending), sg.encode(pending)
    L = 0
    for i in range(len(pending)):
        kind = rng.choice([abi.CA_MATCH_ALL, abi.CA_MATCH_RANGE, abi.CA_MATCH_MASK])
        mask = np.array([rng.random() < 0.7 for _ in nodes], np.uint8)
        lo, hi = sorted(rng.sample(range(len(nodes) + 1), 2))
        match = (kind, lo, hi, rng.choice([-1, rng.randrange(len(nodes))]), mask if kind == abi.CA_MATCH_MASK else None)
        if rng.random() < 0.2:
            L = rng.randrange(0, 1000)
        ro = so.backend.fits_any_node(to, i, match, L)
        rg = sg.backend.fits_any_node(tg, i, match, L)
        assert ro == rg, (seed, i, ro, rg)
        L = ro[1]
        if ro[0] >= 0 and rng.random() < 0.5:       # place it: the state moves on
            for s, t in ((so, to), (sg, tg)):
                s.backend.add_pods(t, [i], [ro[0]])


# --------------------------------------------------------------------------
# estimator
# --------------------------------------------------------------------------
@pytest.mark.parametrize("sort", ["bucket", "merge"])
@pytest.mark.parametrize("seed", range(16))
def test_estimate_random(seed, sort, oracle, monkeypatch):
    monkeypatch.setenv("CASIM_SORT", sort)
    rng, nodes, pods, templates, groups = _estimate_inputs(seed)
    table, node_recs, tm, off, pod_idx = _encode_estimate(nodes, pods, templates, groups)
    max_nodes = rng.choice([0, 0, 3, 10])
    L0 = rng.choice([0, 0, 1, 7, 123])
    outs = []
    for b in (oracle.OracleState(), _mirror()):
        b.clear()
        if len(node_recs):
            b.add_nodes(node_recs)
        outs.append(b.estimate(table, off, pod_idx, tm, max_nodes, L0))
    o, g = outs
    assert np.array_equal(o.results, g.results), (seed, o.results, g.results)
    for k in range(len(groups)):
        n = int(o.results[k]["n_scheduled"])
        a = off[k]
        assert np.array_equal(o.sched_pod[a:a + n], g.sched_pod[a:a + n]), (seed, k)
        assert np.array_equal(o.sched_node[a:a + n], g.sched_node[a:a + n]), (seed, k)
    assert o.last_index == g.last_index


def _run_heavy_inputs(seed, n_groups=6):
    """Pending pods drawn from a handful of shapes and repeated, so the sorted streams are
    long runs of identical pods: the run-batched chain (closed-form revolutions, limiter
    and empty-node skips inside a run) against the per-pod oracle."""
    import copy
    rng = random.Random(1000 + seed)
    nodes = [rand_node(rng, f"e{i}") for i in range(rng.randint(0, 4))]
    shapes = []
    for s in range(rng.randint(1, 5)):
        p = rand_pod(rng, f"shape{s}", small=rng.random() < 0.6)
        p.node_name = ""
        if p.affinity is not None:
            for t in p.affinity.required_terms:
                t.match_fields = []
        if rng.random() < 0.7:
            for c in p.containers:
                c.ports = []
        if rng.random() < 0.5:
            p.affinity = None
            p.node_selector = None
        shapes.append(p)
    pods = []
    for s in shapes:
        for r in range(rng.choice([1, 2, 7, 40, 150])):
            q = copy.deepcopy(s)
            q.name = f"{s.name}-{r}"
            pods.append(q)
    rng.shuffle(pods)
    templates = []
    for g in range(n_groups):
        t = rand_node(rng, f"tmpl{g}", big=rng.random() < 0.5)
        if rng.random() < 0.15:
            t.allocatable["cpu"] = k8s_milli(rng.choice([100, 300]))     # template DS pods overcommit it
        ds = [rand_pod(rng, f"ds{g}-{j}", small=True) for j in range(rng.randint(0, 2))]
        for d in ds:
            d.affinity = None
            d.node_selector = None
        templates.append((t, ds))
    groups = [[p for p in pods if rng.random() < 0.8] for _ in range(n_groups)]
    return rng, nodes, pods, templates, groups


def k8s_milli(v):
    from autoscaler_amd.k8s import Quantity
    return Quantity.milli(v)


@pytest.mark.parametrize("nodes", [True, False], ids=["ordinals", "no-ordinals"])
@pytest.mark.parametrize("batch", ["1", "0"])
@pytest.mark.parametrize("seed", range(24))
def test_estimate_runs_random(seed, batch, nodes, oracle, monkeypatch):
    """Run-heavy streams through both chain modes; without node ordinals the closed-form
    revolutions take the count path (no placement list), which these cases pin too."""
    if batch == "0" and not nodes:
        pytest.skip("per-pod chain: ordinals do not change the path")
    monkeypatch.setenv("CASIM_RUN_BATCH", batch)
    rng, nodes_, pods, templates, groups = _run_heavy_inputs(seed)
    table, node_recs, tm, off, pod_idx = _encode_estimate(nodes_, pods, templates, groups)
    max_nodes = rng.choice([0, 0, 1, 2, 5, 40])
    L0 = rng.choice([0, 0, 1, 3, 7, 123])
    outs = []
    for b in (oracle.OracleState(), _mirror()):
        b.clear()
        if len(node_recs):
            b.add_nodes(node_recs)
        if isinstance(b, oracle.OracleState):
            outs.append(b.estimate(table, off, pod_idx, tm, max_nodes, L0))
        else:
            outs.append(b.estimate(table, off, pod_idx, tm, max_nodes, L0, want_nodes=nodes))
    o, g = outs
    assert np.array_equal(o.results, g.results), (seed, o.results, g.results)
    for k in range(len(groups)):
        n = int(o.results[k]["n_scheduled"])
        a = off[k]
        assert np.array_equal(o.sched_pod[a:a + n], g.sched_pod[a:a + n]), (seed, k)
        if nodes:
            assert np.array_equal(o.sched_node[a:a + n], g.sched_node[a:a + n]), (seed, k)
    assert o.last_index == g.last_index


@pytest.mark.parametrize("nodes", [True, False], ids=["ordinals", "no-ordinals"])
@pytest.mark.parametrize("seed", range(16))
def test_estimate_hbm_rows_random(seed, nodes, oracle, monkeypatch):
    """The chain with its new-node rows in per-group HBM slabs (the path of an unlimited
    estimate too large for LDS, forced here on small inputs): identical to the oracle."""
    monkeypatch.setenv("CASIM_CHAIN_GLOBAL", "1")
    rng, nodes_, pods, templates, groups = _run_heavy_inputs(seed)
    table, node_recs, tm, off, pod_idx = _encode_estimate(nodes_, pods, templates, groups)
    max_nodes = rng.choice([0, 0, 2, 40])
    L0 = rng.choice([0, 3, 123])
    o, m = oracle.OracleState(), _mirror()
    for b in (o, m):
        b.clear()
        if len(node_recs):
            b.add_nodes(node_recs)
    ro = o.estimate(table, off, pod_idx, tm, max_nodes, L0)
    g = m.estimate(table, off, pod_idx, tm, max_nodes, L0, want_nodes=nodes)
    assert np.array_equal(ro.results, g.results), (seed, ro.results, g.results)
    for k in range(len(groups)):
        a, n = off[k], int(ro.results[k]["n_scheduled"])
        assert np.array_equal(ro.sched_pod[a:a + n], g.sched_pod[a:a + n]), (seed, k)
        if nodes:
            assert np.array_equal(ro.sched_node[a:a + n], g.sched_node[a:a + n]), (seed, k)
    assert ro.last_index == g.last_index


def test_estimate_unlimited_full_c2():
    """BASELINE C2 with the unlimited limiter (maxNodes = 0, threshold_based_limiter.go:49-52):
    up to 14k new nodes per group, rows in HBM slabs.  Checked against the committed result
    of the CPU restatement (tests/golden/make_c2_unlimited.py; ~2 min of oracle time)."""
    import json
    import os
    import zlib
    with open(os.path.join(os.path.dirname(__file__), "golden", "c2_unlimited.json")) as f:
        ref = json.load(f)
    w = W.c2()
    m = _mirror()
    W.load_estimate(m, w)
    g = m.estimate(w.table, w.group_off, w.pod_idx, w.templates, 0, 0, want_nodes=False)
    assert g.last_index == ref["last_index"]
    for k, rg in enumerate(ref["groups"]):
        r = g.results[k]
        for f in ("node_count", "n_scheduled", "nodes_added", "last_index_in", "last_index_out", "status", "evals"):
            assert int(r[f]) == rg[f], (k, f, int(r[f]), rg[f])
        a, n = int(w.group_off[k]), rg["n_scheduled"]
        assert zlib.crc32(np.ascontiguousarray(g.sched_pod[a:a + n], np.int32).tobytes()) == rg["sched_crc32"], k


@pytest.mark.parametrize("seed", range(8))
def test_estimate_heavy_first_split(seed, oracle, monkeypatch):
    """G >= 8 groups: the heavy groups sort and chain first on the main stream, the rest
    on a second stream (plan map rebuilt when max_nodes changes); identical to the oracle
    with and without the split, with and without node ordinals."""
    rng, nodes, pods, templates, groups = _run_heavy_inputs(seed, n_groups=16)
    table, node_recs, tm, off, pod_idx = _encode_estimate(nodes, pods, templates, groups)
    o = oracle.OracleState()
    m = _mirror()
    for b in (o, m):
        b.clear()
        if len(node_recs):
            b.add_nodes(node_recs)
    for split in ("1", "0"):
        if split == "0":
            monkeypatch.setenv("CASIM_NO_SPLIT", "1")
        with native.EstimatePlan(m, table, off, pod_idx, tm) as plan:
            for max_nodes in (rng.choice([0, 3, 40]), rng.choice([1, 5, 100])):
                L0 = rng.choice([0, 1, 7, 123])
                ro = o.estimate(table, off, pod_idx, tm, max_nodes, L0)
                for want in (True, False):
                    g = plan.run(max_nodes, L0, want_nodes=want)
                    assert np.array_equal(ro.results, g.results), (seed, split, max_nodes, want)
                    assert ro.last_index == g.last_index
                    for k in range(len(groups)):
                        if int(ro.results[k]["status"]) != 0:
                            continue
                        a, n = off[k], int(ro.results[k]["n_scheduled"])
                        assert np.array_equal(ro.sched_pod[a:a + n], g.sched_pod[a:a + n]), (seed, k)
                        if want:
                            assert np.array_equal(ro.sched_node[a:a + n], g.sched_node[a:a + n]), (seed, k)


@pytest.mark.parametrize("name,w", [
    ("C1", W.c1()),
    ("C2-small", W.c2(n_pods=4000, n_groups=12, n_existing=50)),
    ("C2-unlimited", W.c2(n_pods=1500, n_groups=8, n_existing=20, max_nodes=0)),
    ("C2-medium", W.c2(n_pods=20000, n_groups=20, n_existing=300)),
])
@pytest.mark.parametrize("batch,sort,rows", [("1", "bucket", "lds"), ("0", "bucket", "lds"), ("1", "merge", "lds"),
                                             ("1", "bucket", "hbm"), ("0", "bucket", "hbm")])
def test_estimate_workloads(name, w, batch, sort, rows, oracle, monkeypatch):
    monkeypatch.setenv("CASIM_RUN_BATCH", batch)
    monkeypatch.setenv("CASIM_SORT", sort)
    if rows == "hbm":
        monkeypatch.setenv("CASIM_CHAIN_GLOBAL", "1")
    outs = []
    for b in (oracle.OracleState(), _mirror()):
        W.load_estimate(b, w)
        outs.append(b.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 5))
    o, g = outs
    assert np.array_equal(o.results, g.results)
    assert np.array_equal(o.sched_pod, g.sched_pod)
    assert np.array_equal(o.sched_node, g.sched_node)
    assert o.last_index == g.last_index
    if name == "C1":
        assert int(g.results[0]["node_count"]) == 125 and int(g.results[0]["n_scheduled"]) == 1000


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("stream", ["runs", "radix"])
def test_estimate_decoupled_static_filters(seed, stream, oracle, monkeypatch):
    """Uniform classes with taints, tolerations, selectors, node affinity, host ports and
    extended resources (_run_heavy_inputs: a few pod shapes, each repeated): the decoupled
    stream from per-class counts (k_run_table's per-class static bits against every
    template, non-batchable classes as single pods) and from the radix passes, against the
    Go-order oracle with and without run batching."""
    monkeypatch.setenv("CASIM_RUNS_STREAM", "1" if stream == "runs" else "0")
    rng, nodes_, pods, templates, groups = _run_heavy_inputs(seed, n_groups=8)
    table, node_recs, tm, off, pod_idx = _encode_estimate(nodes_, pods, templates, groups)
    max_nodes = rng.choice([0, 2, 40])
    L0 = rng.choice([0, 3, 77])
    o = oracle.OracleState()
    o.clear()
    if len(node_recs):
        o.add_nodes(node_recs)
    ro = o.estimate(table, off, pod_idx, tm, max_nodes, L0)
    m = _mirror()
    m.clear()
    if len(node_recs):
        m.add_nodes(node_recs)
    for batch in ("1", "0"):
        monkeypatch.setenv("CASIM_RUN_BATCH", batch)
        with native.EstimatePlan(m, table, off, pod_idx, tm) as plan:
            g = plan.run(max_nodes, L0, want_nodes=True)
            assert np.array_equal(ro.results, g.results) and ro.last_index == g.last_index, (seed, batch)
            for k in range(len(groups)):
                if int(ro.results[k]["status"]) != 0:
                    continue
                a, n = off[k], int(ro.results[k]["n_scheduled"])
                assert np.array_equal(ro.sched_pod[a:a + n], g.sched_pod[a:a + n]), (seed, batch, k)
                assert np.array_equal(ro.sched_node[a:a + n], g.sched_node[a:a + n]), (seed, batch, k)
            h = plan.run_u16(max_nodes, L0) if len(table) <= 65535 else None
            if h is not None:
                assert np.array_equal(ro.results, h.results)


@pytest.mark.parametrize("shapes", [300, 3000, 6000])
def test_estimate_many_score_classes(shapes, oracle):
    """Random (cpu, mem) shapes: > 256 score classes take two radix passes, > 4096 take the
    comparison sort; every output in Go sort.Slice order (the oracle's default) — ties
    between shapes of equal float64 score included."""
    w = W.c2(n_pods=8000, n_groups=10, n_existing=30, pods_per_controller=1, n_random_shapes=shapes, seed=shapes)
    outs = []
    for b in (oracle.OracleState(), _mirror()):
        W.load_estimate(b, w)
        outs.append(b.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 3))
    o, g = outs
    assert np.array_equal(o.results, g.results)
    assert np.array_equal(o.sched_pod, g.sched_pod)
    assert np.array_equal(o.sched_node, g.sched_node)
    assert o.last_index == g.last_index


def test_estimate_full_c2_parity(oracle):
    """BASELINE configs[1] at full size (50k pods x 100 groups): bit-exact vs the oracle,
    through ca_estimate_batch and through a plan publishing into page-locked memory."""
    w = W.c2()
    outs = []
    for b in (oracle.OracleState(), _mirror()):
        W.load_estimate(b, w)
        outs.append(b.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 0))
    o, g = outs
    assert np.array_equal(o.results, g.results)
    assert np.array_equal(o.sched_pod, g.sched_pod)
    assert np.array_equal(o.sched_node, g.sched_node)
    assert o.last_index == g.last_index
    m = _mirror()
    W.load_estimate(m, w)
    with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
        for _ in range(2):
            p = plan.run(w.max_nodes, 0, want_nodes=False)
            assert np.array_equal(o.results, p.results)
            assert np.array_equal(o.sched_pod, p.sched_pod)
            assert o.last_index == p.last_index
            d = plan.run(w.max_nodes, 0, device_results=True)        # results left in HBM (bench)
            assert np.array_equal(o.results, d.results)
            assert o.last_index == d.last_index
            assert np.array_equal(o.sched_pod, plan.fetch())
            h = plan.run_u16(w.max_nodes, 0)                           # 16-bit ids (bench headline)
            assert np.array_equal(o.results, h.results)
            assert o.last_index == h.last_index
            assert np.array_equal(o.sched_pod, np.where(h.sched_pod == 0xFFFF, -1, h.sched_pod.astype(np.int32)))


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("decouple", ["1", "radix", "0"], ids=["decoupled", "decoupled-radix", "coupled"])
def test_estimate_go_order_decoupled(seed, decouple, oracle, monkeypatch):
    """Uniform score classes (C2's catalog: every class's pods identical but for their
    controller): the chains run on the stable class order while Go's sort.Slice ids are
    computed beside them (CASIM_GO_DECOUPLE=0: the Go sort ahead of the stream).  The
    decoupled stream comes from per-class counts (k_run_table), or with
    CASIM_RUNS_STREAM=0 from the radix passes.  All give the Go-order oracle's pod lists in
    every output mode, with progressive publishing (64-output chunks), lastIndex
    speculation rounds (existing nodes) and limiter cuts."""
    monkeypatch.setenv("CASIM_GO_DECOUPLE", "0" if decouple == "0" else "1")
    monkeypatch.setenv("CASIM_RUNS_STREAM", "0" if decouple == "radix" else "1")
    monkeypatch.setenv("CASIM_PUB_CHUNK", "64" if seed % 2 else "4096")
    w = W.c2(n_pods=6000 + 1000 * seed, n_groups=6 + seed, n_existing=(0, 20, 200)[seed % 3],
             max_nodes=(1000, 0, 7)[seed % 3], seed=100 + seed)
    o = oracle.OracleState()
    W.load_estimate(o, w)
    L0 = (0, 5, 77)[seed % 3]
    ro = o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, L0)
    m = _mirror()
    W.load_estimate(m, w)
    with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
        for _ in range(2):
            g = plan.run(w.max_nodes, L0, want_nodes=True)
            assert np.array_equal(ro.results, g.results) and ro.last_index == g.last_index
            assert np.array_equal(ro.sched_pod, g.sched_pod) and np.array_equal(ro.sched_node, g.sched_node)
            p = plan.run(w.max_nodes, L0, want_nodes=False)
            assert np.array_equal(ro.sched_pod, p.sched_pod)
            d = plan.run(w.max_nodes, L0, device_results=True)
            assert np.array_equal(ro.results, d.results)
            assert np.array_equal(ro.sched_pod, plan.fetch())
            h = plan.run_u16(w.max_nodes, L0)
            assert np.array_equal(ro.sched_pod, np.where(h.sched_pod == 0xFFFF, -1, h.sched_pod.astype(np.int32)))
            plan.set_phase_timing(False)
            h = plan.run_u16(w.max_nodes, L0)
            plan.set_phase_timing(True)
            assert np.array_equal(ro.results, h.results) and ro.last_index == h.last_index
            assert np.array_equal(ro.sched_pod, np.where(h.sched_pod == 0xFFFF, -1, h.sched_pod.astype(np.int32)))


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("decouple", ["1", "0"], ids=["auto", "coupled"])
def test_estimate_go_order_cross_class_ties(seed, decouple, oracle, monkeypatch):
    """Uniform score classes whose float64 scores tie ACROSS classes on the templates
    (estgen.tied_workload: (1000m, 1Gi), (500m, 3Gi) and (250m, 4Gi) all score 0.3125 on a
    4000m / 16Gi template).  k_class_rank gives them one dense rank and Go's pdqsort mixes
    their pods differently from list position, so the chains must not run on the stable
    order: the plan takes the coupled path (stats()["decoupled"] is False) and matches the
    Go-order oracle in every output mode (binpacking_estimator.go:72-74)."""
    from estgen import tied_workload
    monkeypatch.setenv("CASIM_GO_DECOUPLE", decouple)
    monkeypatch.setenv("CASIM_PUB_CHUNK", "64" if seed % 2 else "4096")
    w, shape_of = tied_workload(seed)
    o = oracle.OracleState()
    W.load_estimate(o, w)
    L0 = (0, 5, 77)[seed % 3]
    ro = o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, L0)
    # the hazard is real on this input: Go's order puts other classes at some sorted
    # positions than the stable order (what a decoupled run would have got wrong)
    o.set_sort_mode("stable")
    rs = o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, L0)
    o.set_sort_mode("go")
    cls_go = np.where(ro.sched_pod >= 0, shape_of[np.maximum(ro.sched_pod, 0)], -1)
    cls_st = np.where(rs.sched_pod >= 0, shape_of[np.maximum(rs.sched_pod, 0)], -1)
    assert not (np.array_equal(cls_go, cls_st) and np.array_equal(ro.results, rs.results))
    m = _mirror()
    W.load_estimate(m, w)
    with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
        for _ in range(2):
            g = plan.run(w.max_nodes, L0, want_nodes=True)
            assert np.array_equal(ro.results, g.results) and ro.last_index == g.last_index
            assert np.array_equal(ro.sched_pod, g.sched_pod) and np.array_equal(ro.sched_node, g.sched_node)
            p = plan.run(w.max_nodes, L0, want_nodes=False)
            assert not plan.stats()["decoupled"]
            assert np.array_equal(ro.results, p.results) and np.array_equal(ro.sched_pod, p.sched_pod)
            d = plan.run(w.max_nodes, L0, device_results=True)
            assert np.array_equal(ro.results, d.results)
            assert np.array_equal(ro.sched_pod, plan.fetch())
            h = plan.run_u16(w.max_nodes, L0)
            assert not plan.stats()["decoupled"]
            assert np.array_equal(ro.results, h.results) and ro.last_index == h.last_index
            assert np.array_equal(ro.sched_pod, np.where(h.sched_pod == 0xFFFF, -1, h.sched_pod.astype(np.int32)))
    b = m.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, L0)      # ca_estimate_batch
    assert np.array_equal(ro.results, b.results) and ro.last_index == b.last_index
    assert np.array_equal(ro.sched_pod, b.sched_pod) and np.array_equal(ro.sched_node, b.sched_node)


def test_estimate_c2_catalog_takes_decoupled_path(oracle):
    """C2's 64-shape catalog has no cross-class score ties on its templates: the headline
    path stays decoupled (and matches the Go-order oracle)."""
    w = W.c2(n_pods=8000, n_groups=12, n_existing=50, seed=3)
    assert w.meta["cross_shape_score_ties"] == 0
    o = oracle.OracleState()
    W.load_estimate(o, w)
    ro = o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 0)
    m = _mirror()
    W.load_estimate(m, w)
    with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
        h = plan.run_u16(w.max_nodes, 0)
        assert plan.stats()["decoupled"]
        assert np.array_equal(ro.results, h.results)
        assert np.array_equal(ro.sched_pod, np.where(h.sched_pod == 0xFFFF, -1, h.sched_pod.astype(np.int32)))


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("chunk", ["4096", "64"], ids=["chunk4096", "chunk64"])
def test_estimate_plan_publish_random(seed, chunk, oracle, monkeypatch):
    """Zero-copy results (plan, page-locked sched_pod, no node ordinals) on random inputs,
    including unsupported and capacity-limited groups.  With 64-output chunks the chains
    publish most chunks while they still run (progressive tickets)."""
    monkeypatch.setenv("CASIM_PUB_CHUNK", chunk)
    rng, nodes, pods, templates, groups = _run_heavy_inputs(seed)
    table, node_recs, tm, off, pod_idx = _encode_estimate(nodes, pods, templates, groups)
    max_nodes = rng.choice([0, 1, 5, 40])
    L0 = rng.choice([0, 3, 123])
    o = oracle.OracleState()
    o.clear()
    if len(node_recs):
        o.add_nodes(node_recs)
    ro = o.estimate(table, off, pod_idx, tm, max_nodes, L0)
    m = _mirror()
    if len(node_recs):
        m.add_nodes(node_recs)
    with native.EstimatePlan(m, table, off, pod_idx, tm) as plan:
        g = plan.run(max_nodes, L0, want_nodes=False)
        d = plan.run(max_nodes, L0, device_results=True)
        dp = plan.fetch()
        h = plan.run_u16(max_nodes, L0)
        hp = np.where(h.sched_pod == 0xFFFF, -1, h.sched_pod.astype(np.int32))
    assert np.array_equal(ro.results, g.results)
    assert np.array_equal(ro.results, d.results)
    assert np.array_equal(ro.results, h.results)
    for k in range(len(groups)):
        if int(ro.results[k]["status"]) != 0:
            continue
        a, b = off[k], off[k + 1]
        n = int(ro.results[k]["n_scheduled"])
        assert np.array_equal(ro.sched_pod[a:a + n], g.sched_pod[a:a + n]), (seed, k)
        assert (g.sched_pod[a + n:b] == -1).all()
        assert np.array_equal(ro.sched_pod[a:a + n], dp[a:a + n]), (seed, k)
        assert (dp[a + n:b] == -1).all()
        assert np.array_equal(ro.sched_pod[a:a + n], hp[a:a + n]), (seed, k)
        assert (hp[a + n:b] == -1).all()
    assert ro.last_index == g.last_index == d.last_index == h.last_index


@pytest.mark.parametrize("serial", [False, True], ids=["concurrent", "serialised"])
def test_estimate_publisher_bounded(serial, oracle, monkeypatch):
    """HIP does not promise that k_publish and the chains overlap.  With the two kernels
    serialised (CASIM_PUB_SERIAL: the publisher first, on the chains' stream) the publisher
    gives up at its start deadline and the stream-ordered copy delivers the results: same
    answers, latency bounded by the deadline (not the 200 ms dead-chain guard)."""
    import time
    if serial:
        monkeypatch.setenv("CASIM_PUB_SERIAL", "1")
    w = W.c2(n_pods=8000, n_groups=20, n_existing=50)
    o = oracle.OracleState()
    W.load_estimate(o, w)
    ro = o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 0)
    m = _mirror()
    W.load_estimate(m, w)
    with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
        walls = []
        for _ in range(3):
            t = time.perf_counter()
            p = plan.run(w.max_nodes, 0, want_nodes=False)
            walls.append(time.perf_counter() - t)
            assert np.array_equal(ro.results, p.results)
            assert np.array_equal(ro.sched_pod, p.sched_pod)
            assert ro.last_index == p.last_index
            assert plan.stats()["results_path"] == ("publisher_gave_up" if serial else "published")
            h = plan.run_u16(w.max_nodes, 0)
            assert np.array_equal(ro.results, h.results)
            assert np.array_equal(ro.sched_pod, np.where(h.sched_pod == 0xFFFF, -1, h.sched_pod.astype(np.int32)))
            assert plan.stats()["results_path"] == ("publisher_gave_up" if serial else "published")
    assert min(walls) < 0.05, walls          # 2 ms start deadline + the copy, never 200 ms


def test_estimate_publisher_state_across_runs(oracle, monkeypatch):
    """Round 1 of a decoupled run skips k_round_init when the last run's publisher consumed
    and reset every ticket and cleared its control words (ca_estimate_plan::pub_clean).
    One plan alternates clean runs, a run whose publisher gives up (serialised: its tickets
    stay dirty, so the next run re-initialises them) and every output mode, with lastIndex
    inputs that force speculation rounds: the results never change."""
    w = W.c2(n_pods=9000, n_groups=16, n_existing=200, max_nodes=1000, seed=11)
    o = oracle.OracleState()
    W.load_estimate(o, w)
    m = _mirror()
    W.load_estimate(m, w)
    ref = {}
    for L0 in (0, 77):
        ref[L0] = o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, L0)

    def check(r, L0, u16=False):
        ro = ref[L0]
        assert np.array_equal(ro.results, r.results) and ro.last_index == r.last_index
        sp = np.where(r.sched_pod == 0xFFFF, -1, r.sched_pod.astype(np.int32)) if u16 else r.sched_pod
        assert np.array_equal(ro.sched_pod, sp)

    with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
        for it in range(4):
            # phase events off (the bench's timed mode): the host joins the publisher and
            # both chain streams itself instead of queueing the waits on the plan's stream
            plan.set_phase_timing(it % 2 == 1)
            for L0 in (0, 77, 0):
                check(plan.run_u16(w.max_nodes, L0), L0, u16=True)
                assert plan.stats()["decoupled"] and plan.stats()["results_path"] == "published"
            check(plan.run(w.max_nodes, 77, want_nodes=False), 77)
            d = plan.run(w.max_nodes, 0, device_results=True)
            assert np.array_equal(ref[0].results, d.results) and np.array_equal(ref[0].sched_pod, plan.fetch())
            monkeypatch.setenv("CASIM_PUB_SERIAL", "1")
            check(plan.run_u16(w.max_nodes, 77), 77, u16=True)
            assert plan.stats()["results_path"] == "publisher_gave_up"
            monkeypatch.delenv("CASIM_PUB_SERIAL")


def test_estimate_publisher_gives_up_in_round1_only(oracle, monkeypatch):
    """A publisher that gives up in round 1 while a later lastIndex round publishes cleanly
    (CASIM_PUB_SERIAL_R1: serialised in round 1 only): the groups round 1 accepted were
    never written into the caller's buffer by any publisher, so the run must take the
    stream-ordered copy (a give-up in any round decides, not the last round's flag)."""
    w = W.c2(n_pods=9000, n_groups=16, n_existing=200, max_nodes=1000, seed=11)
    o = oracle.OracleState()
    W.load_estimate(o, w)
    m = _mirror()
    W.load_estimate(m, w)
    rounds = []
    with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
        for L0 in (77, 0, 77):
            ro = o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, L0)
            monkeypatch.setenv("CASIM_PUB_SERIAL_R1", "1")
            for u16 in (True, False):
                r = plan.run_u16(w.max_nodes, L0) if u16 else plan.run(w.max_nodes, L0, want_nodes=False)
                st = plan.stats()
                assert np.array_equal(ro.results, r.results) and ro.last_index == r.last_index
                sp = np.where(r.sched_pod == 0xFFFF, -1, r.sched_pod.astype(np.int32)) if u16 else r.sched_pod
                assert np.array_equal(ro.sched_pod, sp), (L0, u16, st)
                assert st["results_path"] == "publisher_gave_up", st
                rounds.append(st["rounds"])
            monkeypatch.delenv("CASIM_PUB_SERIAL_R1")
            r = plan.run_u16(w.max_nodes, L0)                 # and a clean run after it
            assert plan.stats()["results_path"] == "published"
            assert np.array_equal(ro.sched_pod, np.where(r.sched_pod == 0xFFFF, -1, r.sched_pod.astype(np.int32)))
    assert max(rounds) > 1, rounds                            # a later round did run (and published)
    m.close()


@pytest.mark.parametrize("size", ["small", "full"])
def test_estimate_c4_taints_affinity(size, oracle):
    """C4 (taint/toleration + node-affinity heavy): static filters on the templates, per
    group pod lists, bit-exact vs the oracle; the plan path publishes zero-copy."""
    w = W.c4() if size == "full" else W.c4(n_pods=6000, n_groups=16, n_existing=60)
    outs = []
    for b in (oracle.OracleState(), _mirror()):
        W.load_estimate(b, w)
        outs.append(b.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 7))
    o, g = outs
    assert np.array_equal(o.results, g.results)
    assert np.array_equal(o.sched_pod, g.sched_pod)
    assert np.array_equal(o.sched_node, g.sched_node)
    assert o.last_index == g.last_index
    m = _mirror()
    W.load_estimate(m, w)
    with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
        p = plan.run(w.max_nodes, 7, want_nodes=False)
    assert np.array_equal(o.results, p.results) and np.array_equal(o.sched_pod, p.sched_pod)


@pytest.mark.parametrize("n_nodes", [800, 5000])
def test_sweep_c4_taints_affinity(n_nodes, oracle):
    """The sweep over a C4-attributed cluster (taints, labels, selectors, required terms):
    two loops (fresh, then hinted), plan with resident hints vs the oracle."""
    w = W.c4_sweep(n_nodes=n_nodes)
    o = oracle.OracleState()
    W.load_sweep(o, w)
    args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
    o1 = o.find_nodes_to_remove(*args, np.full(len(w.table), -1, np.int32), 0)
    o2 = o.find_nodes_to_remove(*args, o1.hints, o1.last_index)
    m = _mirror()
    W.load_sweep(m, w)
    g1 = m.find_nodes_to_remove(*args, np.full(len(w.table), -1, np.int32), 0)
    assert np.array_equal(o1.results, g1.results) and np.array_equal(o1.dest, g1.dest)
    assert np.array_equal(o1.hints, g1.hints) and o1.last_index == g1.last_index
    m.set_hints(o1.hints)
    with native.RemovalPlan(m, *args) as plan:
        g2 = plan.run(o1.last_index, want_dest=True)
    assert np.array_equal(o2.results, g2.results) and np.array_equal(o2.dest, g2.dest)
    assert o2.last_index == g2.last_index
    assert np.array_equal(m.get_hints(len(w.table)), o2.hints)


def test_estimate_full_c2_properties():
    """Full-size C2 (50k pods x 100 groups): every new node's placements fit the template
    (capacity conservation), scheduled pods are distinct members of their group, counts agree."""
    w = W.c2()
    m = _mirror()
    W.load_estimate(m, w)
    out = m.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 0)
    pods = w.table.pods
    for g in range(len(w.templates)):
        r = out.results[g]
        n = int(r["n_scheduled"])
        a = w.group_off[g]
        sp, sn = out.sched_pod[a:a + n], out.sched_node[a:a + n]
        assert len(set(sp.tolist())) == n
        assert set(sp.tolist()) <= set(w.pod_idx[a:w.group_off[g + 1]].tolist())
        t = w.templates[g]
        free_cpu = t["node"]["alloc_milli_cpu"] - t["used_milli_cpu"]
        free_mem = t["node"]["alloc_memory"] - t["used_memory"]
        cpu = np.bincount(sn, weights=pods["req_milli_cpu"][sp], minlength=int(r["nodes_added"]))
        mem = np.bincount(sn, weights=pods["req_memory"][sp].astype(np.float64), minlength=int(r["nodes_added"]))
        assert (cpu <= free_cpu).all() and (mem <= free_mem * (1 + 1e-12)).all()
        assert int(r["node_count"]) == len(set(sn.tolist()))
        assert int(r["nodes_added"]) <= w.max_nodes


# --------------------------------------------------------------------------
# removal sweep
# --------------------------------------------------------------------------
@pytest.mark.parametrize("mode", ["pipeline", "serial"])
@pytest.mark.parametrize("seed", range(12))
def test_sweep_random(seed, mode, oracle, monkeypatch):
    """mode serial: every candidate in one k_sweep chain launch (CASIM_SWEEP_SERIAL, the
    serial-only calls of the planner's late windows)."""
    if mode == "serial":
        monkeypatch.setenv("CASIM_SWEEP_SERIAL", "1")
    rng, nodes, scheduled, pending = rand_cluster(seed, n_nodes=14, n_pods=40, pods_per_node=4)
    it = Interner(nodes, [p for p, _ in scheduled])
    node_recs = it.encode_nodes(nodes)
    table = it.encode_pods([p for p, _ in scheduled])
    pos = {n.name: i for i, n in enumerate(nodes)}
    node_of = np.array([pos[n] for _, n in scheduled], np.int32)
    C = len(nodes)
    cands = np.array(rng.sample(range(C), rng.randint(1, C)), np.int32)
    mask = np.array([rng.random() < 0.85 for _ in nodes], np.uint8)
    status = np.array([rng.choice([0, 0, 0, abi.CA_UNREMOVABLE_BLOCKED_BY_POD]) for _ in cands], np.int32)
    off, moves = [0], []
    for c in cands:
        ids = [i for i in range(len(scheduled)) if node_of[i] == c and rng.random() < 0.9]
        moves.extend(ids)
        off.append(len(moves))
    hints = np.array([rng.choice([-1, -1, rng.randrange(C)]) for _ in scheduled], np.int32)
    L0 = rng.randrange(0, 3 * C)
    outs = []
    for b in (oracle.OracleState(), _mirror()):
        b.clear()
        b.add_nodes(node_recs)
        b.add_pods(table, np.arange(len(scheduled), dtype=np.int32), node_of)
        outs.append(b.find_nodes_to_remove(cands, mask, status, np.array(off, np.int32), np.array(moves, np.int32),
                                           hints, L0))
    o, g = outs
    assert np.array_equal(o.results, g.results), (seed, o.results, g.results)
    assert np.array_equal(o.dest, g.dest), seed
    assert np.array_equal(o.hints, g.hints), seed
    assert o.last_index == g.last_index


@pytest.mark.parametrize("walk", ["device", "host", "host-chain", "serial"])
@pytest.mark.parametrize("n_nodes", [300, 1500, 5000])
def test_sweep_workload(n_nodes, walk, oracle, monkeypatch):
    """host-chain: the host walk hands every batch to the serial exact chain (one k_sweep
    workgroup walking the candidates in order); serial: serial-only calls."""
    if walk in ("host", "host-chain"):
        monkeypatch.setenv("CASIM_SWEEP_HOST_WALK", "1")
    if walk == "host-chain":
        monkeypatch.setenv("CASIM_SWEEP_FORCE_CHAIN", "1")
    if walk == "serial":
        monkeypatch.setenv("CASIM_SWEEP_SERIAL", "1")
    w = W.c3(n_nodes=n_nodes)
    hints = np.full(len(w.table), -1, np.int32)
    outs = []
    for b in (oracle.OracleState(), _mirror()):
        W.load_sweep(b, w)
        outs.append(b.find_nodes_to_remove(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods,
                                           hints, 0))
    o, g = outs
    assert np.array_equal(o.results, g.results)
    assert np.array_equal(o.dest, g.dest)
    assert np.array_equal(o.hints, g.hints)
    assert o.last_index == g.last_index


@pytest.mark.parametrize("n_nodes", [400, 5000])
def test_removal_plan_resident_hints(n_nodes, oracle):
    """The removal plan (inputs resident in HBM) over two loops: fresh hints, then the
    hints the first loop left in the mirror's resident table — vs the oracle's two
    FindNodesToRemove calls with caller-held hints."""
    w = W.c3(n_nodes=n_nodes)
    o = oracle.OracleState()
    W.load_sweep(o, w)
    args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
    o1 = o.find_nodes_to_remove(*args, np.full(len(w.table), -1, np.int32), 0)
    o2 = o.find_nodes_to_remove(*args, o1.hints, o1.last_index)
    m = _mirror()
    W.load_sweep(m, w)
    m.set_hints(np.full(len(w.table), -1, np.int32))
    with native.RemovalPlan(m, *args) as plan:
        g1 = plan.run(0)
        assert np.array_equal(o1.results, g1.results) and o1.last_index == g1.last_index
        assert np.array_equal(m.get_hints(len(w.table)), o1.hints)
        g2 = plan.run(g1.last_index, want_dest=True)
        assert np.array_equal(o2.results, g2.results) and o2.last_index == g2.last_index
        assert np.array_equal(o2.dest, g2.dest)
        assert np.array_equal(m.get_hints(len(w.table)), o2.hints)
        # caller-held hints through the plan
        h = o1.hints.copy()
        g3 = plan.run(o1.last_index, hints=h, want_dest=True)
        assert np.array_equal(o2.results, g3.results) and np.array_equal(o2.dest, g3.dest)
        assert np.array_equal(h, o2.hints)


def test_sweep_with_hints_second_loop(oracle):
    """A second FindNodesToRemove with the hints of the first (the next loop's case)."""
    w = W.c3(n_nodes=400)
    outs = []
    for b in (oracle.OracleState(), _mirror()):
        W.load_sweep(b, w)
        h = np.full(len(w.table), -1, np.int32)
        r1 = b.find_nodes_to_remove(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods, h, 0)
        r2 = b.find_nodes_to_remove(w.candidates[::-1].copy(), w.dest_mask, w.cand_status[::-1].copy(),
                                    *_reverse_moves(w), r1.hints, r1.last_index)
        outs.append((r1, r2))
    (o1, o2), (g1, g2) = outs
    for o, g in ((o1, g1), (o2, g2)):
        assert np.array_equal(o.results, g.results)
        assert np.array_equal(o.dest, g.dest)
        assert np.array_equal(o.hints, g.hints)
        assert o.last_index == g.last_index


def _reverse_moves(w):
    C = len(w.candidates)
    off, moves = [0], []
    for c in reversed(range(C)):
        moves.extend(w.move_pods[w.move_off[c]:w.move_off[c + 1]].tolist())
        off.append(len(moves))
    return np.array(off, np.int32), np.array(moves, np.int32)


def test_fork_revert_commit_parity(oracle):
    rng, nodes, scheduled, pending = rand_cluster(3, n_nodes=6, n_pods=20)
    so, sg = _both(oracle, nodes, scheduled)
    to, tg = so.encode(pending), sg.encode(pending)
    ops = []
    for step in range(60):
        op = rng.choice(["fork", "add", "add", "revert", "commit", "fits"])
        ops.append(op)
        for s, t in ((so, to), (sg, tg)):
            b = s.backend
            if op == "fork":
                b.fork()
            elif op == "add":
                b.add_pods(t, [step % len(pending)], [step % len(nodes)])
            elif op in ("revert", "commit"):
                try:
                    getattr(b, op)()
                except Exception:
                    pass
        if op == "fits":
            assert so.backend.fits_any_node(to, step % len(pending), None, step) == \
                sg.backend.fits_any_node(tg, step % len(pending), None, step), ops
