"""/snapshotz ingestion: the DebuggingSnapshot JSON
(CA/debuggingsnapshot/debugging_snapshot.go:29-72) parsed into the host model and replayed
into the mirror.  The first two tests restate the reference's own tests
(debugging_snapshot_test.go:30-104); the rest check that a cluster survives
dump -> load unchanged and that a replayed snapshot simulates exactly like the original
(oracle backend on CPU, the HIP mirror on the GPU)."""
import json

import numpy as np
import pytest

from autoscaler_amd import snapshotz as Z
from autoscaler_amd import utilization as U
from autoscaler_amd.clustersnapshot import ClusterSnapshot, NodeInfo
from autoscaler_amd.k8s import Node, Pod
from autoscaler_amd.predicatechecker import SchedulerBasedPredicateChecker
from randgen import rand_cluster


def test_basic_setter_workflow():
    """debugging_snapshot_test.go:30-97: NodeList[0].Node.metadata.name, Pods[0].metadata.name."""
    pod = Pod(name="Pod1", node_name="testNode")
    s = Z.DebuggingSnapshot(NodeList=[Z.ClusterNode(Node(name="testNode"), [pod])])
    parsed = json.loads(Z.dump(s))
    assert isinstance(parsed, dict) and isinstance(parsed["NodeList"], list) and len(parsed["NodeList"]) > 0
    n = parsed["NodeList"][0]
    assert n["Node"]["metadata"]["name"] == "testNode"
    assert isinstance(n["Pods"], list) and n["Pods"][0]["metadata"]["name"] == "Pod1"


def test_empty_data_no_error():
    """debugging_snapshot_test.go:99-104."""
    op = Z.dump(Z.DebuggingSnapshot())
    assert op and json.loads(op)["NodeList"] == []


def _cluster(seed):
    _, nodes, scheduled, pending = rand_cluster(seed, n_nodes=12, n_pods=40, pods_per_node=3)
    by_node = {n.name: [] for n in nodes}
    for p, name in scheduled:
        p.node_name = name
        by_node[name].append(p)
    return nodes, by_node, pending


def _snapshot_json(nodes, by_node, pending) -> bytes:
    s = Z.DebuggingSnapshot(NodeList=[Z.ClusterNode(n, by_node[n.name]) for n in nodes],
                            UnscheduledPodsCanBeScheduled=pending, StartTimestamp="2023-02-01T10:00:00Z",
                            EndTimestamp="2023-02-01T10:00:01.123456789Z",
                            TemplateNodes={"ng-1": Z.ClusterNode(nodes[0], [])})
    return Z.dump(s)


@pytest.mark.parametrize("seed", range(6))
def test_round_trip(seed):
    nodes, by_node, pending = _cluster(seed)
    s = Z.load(_snapshot_json(nodes, by_node, pending))
    assert [repr(c.Node) for c in s.NodeList] == [repr(n) for n in nodes]
    assert [repr(c.Pods) for c in s.NodeList] == [repr(by_node[n.name]) for n in nodes]
    assert repr(s.UnscheduledPodsCanBeScheduled) == repr(pending)
    assert list(s.TemplateNodes) == ["ng-1"] and repr(s.TemplateNodes["ng-1"].Node) == repr(nodes[0])
    assert Z.parse_time(s.EndTimestamp) == pytest.approx(1675245601.123456, abs=1e-6)
    assert Z.load(Z.dump(s)) == s or Z.dump(Z.load(Z.dump(s))) == Z.dump(s)


def test_kubernetes_json_fields():
    """Fields as the API server writes them: quantity strings, RFC 3339 times, affinity."""
    d = {"NodeList": [{"Node": {"metadata": {"name": "n1", "labels": {"zone": "a"}},
                                "spec": {"taints": [{"key": "k", "value": "v", "effect": "NoSchedule"}]},
                                "status": {"allocatable": {"cpu": "3920m", "memory": "15Gi", "pods": "110"}}},
                       "Pods": [{"metadata": {"name": "p", "namespace": "kube-system",
                                              "deletionTimestamp": "2020-12-18T16:50:00Z",
                                              "ownerReferences": [{"kind": "DaemonSet", "name": "ds",
                                                                   "controller": True}]},
                                 "spec": {"nodeName": "n1", "terminationGracePeriodSeconds": 45,
                                          "containers": [{"resources": {"requests": {"cpu": "0.1",
                                                                                     "memory": "128Mi"}},
                                                          "ports": [{"containerPort": 80, "hostPort": 8080}]}],
                                          "affinity": {"nodeAffinity": {
                                              "requiredDuringSchedulingIgnoredDuringExecution": {
                                                  "nodeSelectorTerms": [{"matchExpressions": [
                                                      {"key": "zone", "operator": "In", "values": ["a"]}]}]}}},
                                          "volumes": [{"name": "x", "emptyDir": {}}]}}]}]}
    s = Z.load(json.dumps(d))
    n, p = s.NodeList[0].Node, s.NodeList[0].Pods[0]
    assert n.allocatable["cpu"].milli_value() == 3920 and n.allocatable["memory"].value() == 15 << 30
    assert n.taints[0].effect == "NoSchedule" and n.labels == {"zone": "a"}
    assert p.containers[0].requests["cpu"].milli_value() == 100
    assert p.containers[0].requests["memory"].value() == 128 << 20
    assert p.containers[0].ports[0].host_port == 8080 and p.volumes == ["emptyDir"]
    assert p.affinity.required_terms[0].match_expressions[0].values == ["a"]
    assert p.deletion_timestamp == 1608310200.0 and p.termination_grace_period_seconds == 45
    assert U.is_daemonset_pod(p)
    assert s.UnscheduledPodsCanBeScheduled == [] and s.TemplateNodes == {}


def _replay_fits(backend_factory, nodes, by_node, pending, replayed: bool):
    if replayed:
        s = Z.load(_snapshot_json(nodes, by_node, pending))
        snap, pending = Z.cluster_snapshot(s, backend_factory()), s.UnscheduledPodsCanBeScheduled
    else:
        snap = ClusterSnapshot(backend_factory())
        for n in nodes:
            snap.AddNodeWithPods(n, list(by_node[n.name]))
    pc = SchedulerBasedPredicateChecker()
    out = []
    for p in pending:                                  # FitsAnyNode + AddPod, as the estimator loop
        name, err = pc.FitsAnyNode(snap, p)
        out.append(name if err is None else None)
        if err is None:
            snap.AddPod(p, name)
    return out, pc.last_index, pc.evals


@pytest.mark.parametrize("seed", range(4))
def test_replay_oracle(seed, oracle_lib):
    nodes, by_node, pending = _cluster(seed)
    a = _replay_fits(oracle_lib.OracleState, nodes, by_node, pending, False)
    b = _replay_fits(oracle_lib.OracleState, *_cluster(seed), True)
    assert a == b and any(x is not None for x in a[0])


def test_replay_utilization_rows(oracle_lib):
    nodes, by_node, pending = _cluster(3)
    s = Z.load(_snapshot_json(nodes, by_node, pending))
    a = U.build_table([NodeInfo(n, by_node[n.name]) for n in nodes], [None] * len(nodes))
    b = U.build_table([NodeInfo(c.Node, c.Pods) for c in s.NodeList], [None] * len(nodes))
    for x, y in zip(a, b):
        assert x.tobytes() == y.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_replay_gpu(seed, oracle_lib):
    from autoscaler_amd import native
    nodes, by_node, pending = _cluster(seed)
    ref = _replay_fits(oracle_lib.OracleState, nodes, by_node, pending, False)
    got = _replay_fits(lambda: native.Mirror(0), *_cluster(seed), True)
    assert got == ref
