"""Kernel scope: out-of-scope inputs are rejected, never simulated;
the batch prefix protocol; RemoveNode; the drain-policy fixes of ADVICE r1.

Every scenario runs on the CPU checker (oracle) here and through libcasim on the
GPU (`-m gpu`): both must reject the same inputs and agree on every prefix result.
"""
import numpy as np
import pytest

from autoscaler_amd import abi, k8s
from autoscaler_amd.clustersnapshot import ClusterSnapshot, NodeInfo
from autoscaler_amd.drain import NodeDeleteOptions, get_pods_to_move, is_pod_long_terminating, is_pod_terminal
from autoscaler_amd.estimator import (BinpackingNodeEstimator, ThresholdBasedEstimationLimiter, UnsupportedByKernels,
                                      estimate_batch)
from autoscaler_amd.intern import Interner
from autoscaler_amd.podlistprocessor import FilterOutSchedulablePodListProcessor
from autoscaler_amd.predicatechecker import SchedulerBasedPredicateChecker
from autoscaler_amd.scope import out_of_scope_reason
from autoscaler_amd.simulator import RemovalSimulator

BACKENDS = ["oracle", pytest.param("native", marks=pytest.mark.gpu)]


def backend(name):
    if name == "oracle":
        import pyoracle
        return pyoracle.OracleState()
    from autoscaler_amd import native
    return native.Mirror(0)


def pod(name, cpu=100, mem=100 << 20, owner=None, node=""):
    p = k8s.build_test_pod(name, cpu, mem)
    if owner:
        p.owner_refs = [k8s.OwnerReference("ReplicaSet", owner, owner)]
    p.node_name = node
    return p


def spread(p, when="DoNotSchedule"):
    p.topology_spread.append(k8s.TopologySpreadConstraint(1, "kubernetes.io/hostname", when, {"app": "x"}))
    return p


def anti(p):
    p.affinity = k8s.Affinity(pod_affinity=True, required_anti_affinity=True)
    return p


# ---------------------------------------------------------------------------
# the classifier
# ---------------------------------------------------------------------------
def test_classifier():
    assert out_of_scope_reason(pod("a")) is None
    assert out_of_scope_reason(spread(pod("a"), "ScheduleAnyway")) is None      # soft constraints: no Filter
    assert "PodTopologySpread" in out_of_scope_reason(spread(pod("a")))
    p = pod("a")
    p.affinity = k8s.Affinity(pod_affinity=True)                                 # preferred terms only
    assert out_of_scope_reason(p) is None
    assert "InterPodAffinity" in out_of_scope_reason(anti(pod("a")))
    p.affinity = k8s.Affinity(pod_affinity=True, required_pod_affinity=True)
    assert "InterPodAffinity" in out_of_scope_reason(p)
    for v in ("emptyDir", "hostPath", "configMap", "secret", "projected", "downwardAPI"):
        q = pod("v")
        q.volumes = [v]
        assert out_of_scope_reason(q) is None, v
    for v in ("persistentVolumeClaim", "ephemeral", "gcePersistentDisk", "awsElasticBlockStore", "csi", "rbd"):
        q = pod("v")
        q.volumes = ["emptyDir", v]
        assert "volume" in out_of_scope_reason(q), v
    flags = Interner().encode_pods([pod("a"), spread(pod("b")), anti(pod("c"))]).pods["flags"]
    assert [bool(f & abi.CA_POD_OUT_OF_SCOPE) for f in flags] == [False, True, True]
    assert [bool(f & abi.CA_POD_REQUIRED_ANTI_AFFINITY) for f in flags] == [False, False, True]


# ---------------------------------------------------------------------------
# rejection through the facades
# ---------------------------------------------------------------------------
def _snap(b, nodes=3):
    s = ClusterSnapshot(backend(b))
    s.AddNodes([k8s.build_test_node(f"n{i}", 4000, 8 << 30) for i in range(nodes)])
    return s


@pytest.mark.parametrize("b", BACKENDS)
def test_out_of_scope_pod_rejected(b):
    s = _snap(b)
    pc = SchedulerBasedPredicateChecker()
    q = pod("pvc")
    q.volumes = ["persistentVolumeClaim"]
    with pytest.raises(UnsupportedByKernels):
        pc.FitsAnyNode(s, q)
    with pytest.raises(UnsupportedByKernels):
        pc.CheckPredicates(s, spread(pod("t")), "n0")
    assert pc.last_index == 0 and pc.FitsAnyNode(s, pod("ok"))[0] == "n0"
    est = BinpackingNodeEstimator(pc, s, ThresholdBasedEstimationLimiter(0))
    with pytest.raises(UnsupportedByKernels):
        est.Estimate([pod("a"), anti(pod("b"))], NodeInfo(k8s.build_test_node("t", 1000, 1 << 30), []))
    # a template whose DaemonSet pods carry required anti-affinity: the group is out of scope
    with pytest.raises(UnsupportedByKernels):
        est.Estimate([pod("a")], NodeInfo(k8s.build_test_node("t", 1000, 1 << 30), [anti(pod("ds"))]))
    fos = FilterOutSchedulablePodListProcessor(pc)
    with pytest.raises(UnsupportedByKernels):
        fos.Process(s, [pod("a"), spread(pod("b"))])
    assert s.List()[0].pods == []                                    # nothing was placed


@pytest.mark.parametrize("b", BACKENDS)
def test_anti_affinity_in_cluster_blocks_everything(b):
    s = _snap(b)
    s.AddPod(anti(pod("x", owner="rs")), "n1")
    assert s.backend.scope_blockers() == 1
    pc = SchedulerBasedPredicateChecker()
    with pytest.raises(UnsupportedByKernels):
        pc.FitsAnyNode(s, pod("ok"))
    with pytest.raises(UnsupportedByKernels):
        BinpackingNodeEstimator(pc, s, ThresholdBasedEstimationLimiter(0)).Estimate(
            [pod("a")], NodeInfo(k8s.build_test_node("t", 1000, 1 << 30), []))
    with pytest.raises(UnsupportedByKernels):
        FilterOutSchedulablePodListProcessor(pc).Process(s, [pod("a")])
    sim = RemovalSimulator(None, s, pc)
    with pytest.raises(UnsupportedByKernels):
        sim.FindNodesToRemove(["n0"], s.node_names())
    # the count follows the snapshot: fork + remove + revert, then remove for good
    s.Fork()
    s.RemovePod("default", "x", "n1")
    assert s.backend.scope_blockers() == 0
    s.Revert()
    assert s.backend.scope_blockers() == 1
    s.RemovePod("default", "x", "n1")
    assert s.backend.scope_blockers() == 0
    assert pc.FitsAnyNode(s, pod("ok"))[0] == "n0"


# ---------------------------------------------------------------------------
# prefix protocol of the batch entry points (include/casim.h kernel scope)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("b", BACKENDS)
def test_estimate_prefix_protocol(b):
    s = _snap(b, nodes=2)
    s.AddPod(pod("big0", 3900), "n0")
    s.AddPod(pod("big1", 3900), "n1")
    tmpl = NodeInfo(k8s.build_test_node("t", 1000, 4 << 30), [])
    groups = [([pod(f"a{i}", 300) for i in range(7)], tmpl),
              ([pod("b0", 300), spread(pod("b1", 300))], tmpl),
              ([pod(f"c{i}", 300) for i in range(5)], tmpl)]
    all_pods = [p for g, _ in groups for p in g]
    s.ensure(pods=all_pods, templates=[(tmpl.node, [])])
    table = s.interner.encode_pods(all_pods)
    tm = np.stack([s.interner.encode_template(tmpl.node, [])] * 3)
    off = np.array([0, 7, 9, 14], np.int32)
    out = s.backend.estimate(table, off, np.arange(14, dtype=np.int32), tm, 0, 5)
    st = out.results["status"].tolist()
    assert st == [abi.CA_OK, abi.CA_EUNSUPPORTED, abi.CA_ENOTRUN]
    assert out.results[0]["node_count"] == 3 and out.results[0]["n_scheduled"] == 7
    # lastIndex: the value group 1 starts from (group 0's output); group 2 reports it too
    assert out.last_index == int(out.results[0]["last_index_out"]) == int(out.results[1]["last_index_in"])
    assert int(out.results[2]["last_index_in"]) == out.last_index and int(out.results[2]["n_scheduled"]) == 0
    # the caller resumes after the out-of-scope group with the remaining groups
    out2 = s.backend.estimate(table, np.array([0, 5], np.int32), np.arange(9, 14, dtype=np.int32), tm[:1], 0,
                              out.last_index)
    assert out2.results["status"].tolist() == [abi.CA_OK] and out2.results[0]["n_scheduled"] == 5


@pytest.mark.parametrize("b", BACKENDS)
@pytest.mark.parametrize("plan", [False, True], ids=["call", "plan"])
def test_sweep_prefix_protocol(b, plan):
    if plan and b == "oracle":
        pytest.skip("removal plans are a libcasim feature")
    s = _snap(b, nodes=5)
    s.AddPod(pod("p0", 500, owner="rs"), "n0")
    q = pod("p1", 500, owner="rs")
    q.volumes = ["persistentVolumeClaim"]
    s.AddPod(q, "n1")
    s.AddPod(pod("p2", 500, owner="rs"), "n2")
    ids = [pid for n in ("n0", "n1", "n2") for _, pid in s.pod_ids(n)]
    cand = np.array([0, 1, 2], np.int32)
    mask = np.ones(5, np.uint8)
    off = np.array([0, 1, 2, 3], np.int32)
    moves = np.array(ids, np.int32)
    hints = np.full(3, -1, np.int32)
    if plan:
        from autoscaler_amd import native
        with native.RemovalPlan(s.backend, cand, mask, None, off, moves) as pl:
            out = pl.run(7, hints, want_dest=True)
    else:
        out = s.backend.find_nodes_to_remove(cand, mask, None, off, moves, hints, 7)
    assert out.results["reason"].tolist() == [0, abi.CA_UNREMOVABLE_OUT_OF_SCOPE, abi.CA_UNREMOVABLE_NOT_RUN]
    assert out.results["removable"].tolist() == [1, 0, 0]
    assert out.dest[0] >= 0 and out.dest[1] == -1 and out.dest[2] == -1
    assert out.last_index == int(out.results[1]["last_index_in"]) == int(out.results[2]["last_index_in"])
    with pytest.raises(UnsupportedByKernels):
        RemovalSimulator(None, s, SchedulerBasedPredicateChecker()).FindNodesToRemove(
            ["n0", "n1", "n2"], s.node_names())


@pytest.mark.parametrize("b", BACKENDS)
def test_check_templates_unsupported_pairs(b):
    s = _snap(b, nodes=1)
    pods = [pod("a"), spread(pod("b")), pod("c")]
    tn = k8s.build_test_node("t", 1000, 1 << 30)
    s.ensure(pods=pods + [anti(pod("ds"))], templates=[(tn, [])])
    table = s.interner.encode_pods(pods)
    tm = np.stack([s.interner.encode_template(tn, []), s.interner.encode_template(tn, [anti(pod("ds"))])])
    out = s.backend.check_templates(table, np.arange(3, dtype=np.int32), tm)
    assert out["type"].tolist() == [[abi.CA_PRED_OK, abi.CA_PRED_UNSUPPORTED, abi.CA_PRED_OK],
                                    [abi.CA_PRED_UNSUPPORTED] * 3]


# ---------------------------------------------------------------------------
# RemoveNode (clustersnapshot.go:38, delta.go:150-186)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("b", BACKENDS)
def test_remove_node(b):
    s = _snap(b, nodes=4)
    for i, c in enumerate((900, 400, 3900, 3900)):
        s.AddPod(pod(f"p{i}", c), f"n{i}")
    pc = SchedulerBasedPredicateChecker()
    big = pod("big", 3000)
    assert pc.FitsAnyNode(s, big)[0] == "n0"            # 3100 free
    s.Fork()
    s.RemoveNode("n0")
    assert s.node_names() == ["n1", "n2", "n3"]
    pc.last_index = 0
    assert pc.FitsAnyNode(s, big)[0] == "n1"            # positions shifted: n1 is first now
    assert s.backend.pod_node(0) == -1 and s.backend.pod_node(1) == 0
    s.Revert()
    assert s.node_names() == ["n0", "n1", "n2", "n3"]
    assert s.backend.pod_node(0) == 0 and s.backend.pod_node(3) == 3
    pc.last_index = 0
    assert pc.FitsAnyNode(s, big)[0] == "n0"
    s.RemoveNode("n2")                                  # unforked: permanent
    assert s.node_names() == ["n0", "n1", "n3"] and s.backend.node_count() == 3
    assert s.backend.node_pods(2) == [3]
    with pytest.raises(KeyError):
        s.RemoveNode("n2")


@pytest.mark.gpu
def test_remove_node_resident_hints():
    """Resident hints follow the positions; a hint to the removed node comes back on Revert."""
    from autoscaler_amd import native
    m = native.Mirror(0)
    recs = np.zeros(4, abi.NODE_DTYPE)
    recs["alloc_milli_cpu"] = 1000
    recs["alloc_pods"] = 10
    m.add_nodes(recs)
    m.set_hints(np.zeros(0, np.int32))
    t = Interner().encode_pods([pod("a"), pod("b"), pod("c")])
    m.add_pods(t, [0, 1, 2], [0, 1, 2])
    m.set_hints(np.array([3, 1, 2], np.int32))
    m.fork()
    m.remove_node(1)
    h = m.get_hints(3)
    assert h[0] == 2 and h[1] < 0 and h[2] == 1
    m.revert()
    assert m.get_hints(3).tolist() == [3, 1, 2]
    # two removals at the same position (node 1, then node 2 that shifted into
    # position 1) keep distinct codes; each Revert restores exactly its own node's hints
    m.fork()
    m.remove_node(1)
    m.remove_node(1)
    h = m.get_hints(3)
    assert h[0] == 1 and h[1] < 0 and h[2] < 0 and h[1] != h[2]
    m.revert()
    assert m.get_hints(3).tolist() == [3, 1, 2]
    m.fork()
    m.remove_node(1)
    m.fork()
    m.remove_node(1)
    m.revert()                                   # only the second removal (node 2) comes back
    h = m.get_hints(3)
    assert h[0] == 2 and h[1] < 0 and h[2] == 1
    m.revert()
    assert m.get_hints(3).tolist() == [3, 1, 2]


# ---------------------------------------------------------------------------
# drain policy (IsPodLongTerminating grace period, isPodTerminal,
# IsDaemonSetPod annotation)
# ---------------------------------------------------------------------------
def test_long_terminating_uses_grace_period():
    p = pod("p", owner="rs")
    p.deletion_timestamp = 1000.0
    assert not is_pod_long_terminating(p, 1000.0 + 45)           # default grace 30 s + 30 s threshold
    assert not is_pod_long_terminating(p, 1000.0 + 60)           # strictly before
    assert is_pod_long_terminating(p, 1000.0 + 60.5)
    p.termination_grace_period_seconds = 0
    assert is_pod_long_terminating(p, 1000.0 + 30.5)
    # FindEmptyNodesToRemove: a pod deleted 45 s ago with the default grace still counts
    unrep = pod("u")
    unrep.deletion_timestamp = 1000.0
    pods, _, block, err = get_pods_to_move([unrep], NodeDeleteOptions(), None, [], 1045.0)
    assert err is not None and block.pod is unrep
    assert get_pods_to_move([unrep], NodeDeleteOptions(), None, [], 1061.0)[3] is None


def test_pod_terminal_restart_policy():
    p = pod("p")
    p.phase = "Succeeded"
    assert not is_pod_terminal(p)                                # restartPolicy Always
    p.restart_policy = "OnFailure"
    assert is_pod_terminal(p)
    p.restart_policy = "Always"
    p.phase = "Failed"
    assert is_pod_terminal(p)
    # a Succeeded, unreplicated pod with restartPolicy Always blocks the drain
    q = pod("q")
    q.phase = "Succeeded"
    assert get_pods_to_move([q], NodeDeleteOptions(), None, [])[3] is not None


def test_daemonset_annotation():
    p = pod("ds")
    p.annotations[k8s.DAEMONSET_POD_ANNOTATION] = "true"
    pods, ds, block, err = get_pods_to_move([p], NodeDeleteOptions(), None, [])
    assert err is None and pods == [] and ds == [p]
    # drain.go branch order: an annotated ReplicaSet pod is a DaemonSet pod
    q = pod("rs-ds", owner="rs")
    q.annotations[k8s.DAEMONSET_POD_ANNOTATION] = "true"
    pods, ds, block, err = get_pods_to_move([q], NodeDeleteOptions(), None, [])
    assert err is None and pods == [] and ds == [q]
    assert Interner().encode_pods([q]).pods["flags"][0] & abi.CA_POD_DAEMONSET


# ---------------------------------------------------------------------------
# intern widths and the sweep's destination table (verdict r2): a value past a fixed
# width (casim.h) routes exactly the objects that need it to the reference path
# ---------------------------------------------------------------------------
def _taint_snap(b, n_nodes):
    s = ClusterSnapshot(backend(b))
    nodes = []
    for i in range(n_nodes):
        n = k8s.build_test_node(f"n{i}", 4000, 8 << 30)
        n.taints.append(k8s.Taint(f"t{i}", "v", "NoSchedule"))
        nodes.append(n)
    s.AddNodes(nodes)
    return s


@pytest.mark.parametrize("b", BACKENDS)
def test_taint_classes_past_width(b):
    """66 taint classes: 63 interned, 3 share bit 63.  Pods that tolerate none or all of the
    overflow taints are exact; a pod tolerating some of them goes to the reference path."""
    s = _taint_snap(b, 66)
    it = s.interner
    assert len(it.taints) == 63 and len(it.taints.overflow) == 3
    pc = SchedulerBasedPredicateChecker()
    assert not pc.FitsAnyNode(s, pod("plain"))[0]                        # every node tainted
    every = pod("every")
    every.tolerations.append(k8s.Toleration(operator="Exists"))
    pc.last_index = 64
    assert pc.FitsAnyNode(s, every)[0] == "n64"                          # an overflow node, tolerated
    t0 = pod("t0")
    t0.tolerations.append(k8s.Toleration(key="t0", operator="Exists"))
    pc.last_index = 3
    assert pc.FitsAnyNode(s, t0)[0] == "n0"
    some = pod("some")
    some.tolerations.append(k8s.Toleration(key="t65", operator="Exists"))
    table = s.interner.encode_pods([pod("plain"), every, t0, some])
    assert [bool(f & abi.CA_POD_OUT_OF_SCOPE) for f in table.pods["flags"]] == [False, False, False, True]
    with pytest.raises(UnsupportedByKernels):
        pc.FitsAnyNode(s, some)
    # Estimate on a template carrying an overflow taint: the prefix protocol cuts at the group
    # with the partially tolerating pod
    tn = k8s.build_test_node("tmpl", 4000, 8 << 30)
    tn.taints.append(k8s.Taint("t65", "v", "NoSchedule"))
    tmpl = NodeInfo(tn, [])
    est = BinpackingNodeEstimator(pc, s, ThresholdBasedEstimationLimiter(0))
    assert est.Estimate([every], tmpl)[0] == 1
    assert est.Estimate([pod("plain2")], tmpl)[0] == 0
    with pytest.raises(UnsupportedByKernels):
        est.Estimate([every, some], tmpl)


@pytest.mark.parametrize("b", BACKENDS)
def test_extended_resources_past_width(b):
    """9 extended resources: a pod requesting the 9th is out of scope, one requesting the
    1st is simulated, and the 9th on a node's allocatable does not disturb either."""
    s = ClusterSnapshot(backend(b))
    n = k8s.build_test_node("n0", 4000, 8 << 30)
    for r in range(9):
        n.allocatable[f"example.com/r{r}"] = k8s.Quantity(4)
    s.AddNodes([n])
    assert len(s.interner.scalars) == 8 and s.interner.scalars.overflow == {"example.com/r8"}
    pc = SchedulerBasedPredicateChecker()
    first = pod("first")
    first.containers[0].requests["example.com/r0"] = k8s.Quantity(3)
    assert pc.FitsAnyNode(s, first)[0] == "n0"
    too_much = pod("too-much")
    too_much.containers[0].requests["example.com/r0"] = k8s.Quantity(5)
    assert not pc.FitsAnyNode(s, too_much)[0]
    ninth = pod("ninth")
    ninth.containers[0].requests["example.com/r8"] = k8s.Quantity(1)
    with pytest.raises(UnsupportedByKernels):
        pc.FitsAnyNode(s, ninth)


@pytest.mark.parametrize("b", BACKENDS)
def test_candidate_past_destination_table(b):
    """A candidate with more than CA_MAX_MOVED_PODS (128) pods to move is the prefix cut of
    FindNodesToRemove (k_sweep keeps a candidate's destinations in a 128-entry table): the
    candidates before it are simulated, it is CA_UNREMOVABLE_OUT_OF_SCOPE, the rest NOT_RUN."""
    s = ClusterSnapshot(backend(b))
    big = k8s.build_test_node("big", 64000, 64 << 30, pods=200)
    small = k8s.build_test_node("small", 4000, 8 << 30)
    spare = [k8s.build_test_node(f"d{i}", 1000, 8 << 30, pods=1) for i in range(140)]
    s.AddNodes([small, big] + spare + [k8s.build_test_node("last", 4000, 8 << 30)])
    s.AddPod(pod("sp", 100, owner="rs"), "small")
    for i in range(129):                           # 129 pods, each needs a node of its own
        s.AddPod(pod(f"bp{i}", 100, owner="rs"), "big")
    s.AddPod(pod("lp", 100, owner="rs"), "last")
    names = ["small", "big", "last"]
    ids = [[pid for _, pid in s.pod_ids(n)] for n in names]
    cand = np.array([s.position(n) for n in names], np.int32)
    off = np.array([0, 1, 130, 131], np.int32)
    moves = np.array([i for l in ids for i in l], np.int32)
    n_nodes = len(s.node_names())
    out = s.backend.find_nodes_to_remove(cand, np.ones(n_nodes, np.uint8), None, off, moves,
                                         np.full(int(moves.max()) + 1, -1, np.int32), 0)
    assert out.results["reason"].tolist() == [0, abi.CA_UNREMOVABLE_OUT_OF_SCOPE, abi.CA_UNREMOVABLE_NOT_RUN]
    assert out.results["removable"].tolist() == [1, 0, 0]
    assert out.last_index == int(out.results[1]["last_index_in"])
    # 128 pods to move stay in scope
    out = s.backend.find_nodes_to_remove(cand[1:2], np.ones(n_nodes, np.uint8), None, np.array([0, 128], np.int32),
                                         moves[1:129], np.full(int(moves.max()) + 1, -1, np.int32), 0)
    assert out.results["reason"].tolist() != [abi.CA_UNREMOVABLE_OUT_OF_SCOPE]
    with pytest.raises(UnsupportedByKernels):
        RemovalSimulator(None, s, SchedulerBasedPredicateChecker()).FindNodesToRemove(names, s.node_names())
