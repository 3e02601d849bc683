"""Scale-down eligibility: utilization.Calculate
(CA/simulator/utilization/info.go:48-127) and FindEmptyNodesToRemove
(CA/simulator/cluster.go:187-202).

CPU: the oracle (or_node_utilization) against the reference's own TestCalculate
scenarios (CA/simulator/utilization/info_test.go:32-122, same pods, nodes and asserts) and
the empty-node cases of cluster_test.go:39-70.  GPU (marked): libcasim.so's
ca_util_calculate bit-exact (float64 bytes, statuses, verdicts) against the oracle on the
same scenarios, random tables with every edge case, and the full C5 size (15k nodes)."""
import datetime

import numpy as np
import pytest

from autoscaler_amd import abi
from autoscaler_amd import utilization as U
from autoscaler_amd import workloads as W
from autoscaler_amd.clustersnapshot import NodeInfo
from autoscaler_amd.drain import NodeDeleteOptions
from autoscaler_amd.k8s import (OwnerReference, add_gpus_to_node, build_test_node, build_test_pod,
                                request_gpu_for_pod, set_rs_pod, tolerate_gpu_for_pod)

TEST_TIME = datetime.datetime(2020, 12, 18, 17, 0, 0, tzinfo=datetime.timezone.utc).timestamp()
GPU_LABEL, GPU_RESOURCE = "cloud.google.com/gke-accelerator", "nvidia.com/gpu"


def gpu_config_from_node(node):
    """GetGpuConfigFromNode (CA/utils/test/test_utils.go:245-256)."""
    has_label = GPU_LABEL in node.labels
    alloc = node.allocatable.get(GPU_RESOURCE)
    if has_label or (alloc is not None and alloc.milli_value() != 0):
        return U.GpuConfig(GPU_LABEL, node.labels.get(GPU_LABEL, ""), GPU_RESOURCE)
    return None


def info_test_cases():
    """(name, NodeInfo, skipDS, skipMirror, expected utilization or 'error') — info_test.go:32-122."""
    pod = build_test_pod("p1", 100, 200000)
    pod2 = build_test_pod("p2", -1, -1)
    node = build_test_node("node1", 2000, 2000000)
    node2 = build_test_node("node1", 2000, -1)
    ds3 = build_test_pod("p3", 100, 200000)
    ds3.owner_refs = [OwnerReference("DaemonSet", "ds")]
    ds4 = build_test_pod("p4", 100, 200000)
    ds4.owner_refs = [OwnerReference("CustomDaemonSet", "ds")]
    ds4.annotations = {"cluster-autoscaler.kubernetes.io/daemonset-pod": "true"}
    term = build_test_pod("podTerminated", 100, 200000)
    term.deletion_timestamp = TEST_TIME - 600
    mirror = build_test_pod("p4", 100, 200000)
    mirror.annotations = {"kubernetes.io/config.mirror": ""}
    gpu_node = build_test_node("gpu_node", 2000, 2000000)
    add_gpus_to_node(gpu_node, 1)
    gpu_pod = build_test_pod("gpu_pod", 100, 200000)
    request_gpu_for_pod(gpu_pod, 1)
    tolerate_gpu_for_pod(gpu_pod)
    unready = build_test_node("gpu_node", 2000, 2000000)
    unready.labels[GPU_LABEL] = "nvidia-tesla-k80"                  # AddGpuLabelToNode
    return [
        ("basic", NodeInfo(node, [pod, pod, pod2]), False, False, 2.0 / 10),
        ("no-memory", NodeInfo(node2, [pod, pod, pod2]), False, False, "error"),
        ("skip-ds", NodeInfo(node, [pod, pod, pod2, ds3, ds4]), True, False, 2.5 / 10),
        ("count-ds", NodeInfo(node, [pod, pod2, ds3]), False, False, 2.0 / 10),
        ("terminated", NodeInfo(node, [pod, pod, pod2, term]), False, False, 2.0 / 10),
        ("skip-mirror", NodeInfo(node, [pod, pod, pod2, mirror]), False, True, 2.0 / 9.0),
        ("count-mirror", NodeInfo(node, [pod, pod2, mirror]), False, False, 2.0 / 10),
        ("skip-both", NodeInfo(node, [pod, mirror, ds3]), True, True, 1.0 / 8.0),
        ("gpu", NodeInfo(gpu_node, [pod, pod, gpu_pod]), False, False, 1.0),
        ("unready-gpu", NodeInfo(unready, [pod, pod]), False, False, 0.0),
    ]


def _table(cases):
    nis = [c[1] for c in cases]
    return U.build_table(nis, [gpu_config_from_node(n.node) for n in nis])


def _check_expected(name, row, expected):
    if expected == "error":
        assert row["status"] != abi.CA_UTIL_OK, name
    else:
        assert row["status"] == abi.CA_UTIL_OK, name
        if expected == 0.0:
            assert row["utilization"] == 0.0, name
        else:                                                     # assert.InEpsilon(.., 0.01)
            assert abs(row["utilization"] - expected) / abs(expected) <= 0.01, (name, row["utilization"])


@pytest.mark.parametrize("case", range(10))
def test_oracle_info_test_cases(case, oracle_lib):
    cases = info_test_cases()
    name, _, sds, smp, expected = cases[case]
    nodes, off, pods = _table([cases[case]])
    out = oracle_lib.node_utilization(nodes, off, pods, sds, smp, round(TEST_TIME * 1e9))
    _check_expected(name, out[0], expected)


def test_oracle_resource_name_and_error_order(oracle_lib):
    cases = info_test_cases()
    nodes, off, pods = _table(cases)
    out = oracle_lib.node_utilization(nodes, off, pods, False, False, round(TEST_TIME * 1e9))
    assert out[0]["resource"] == abi.CA_UTIL_MEM and out[0]["cpu"] == 0.1 and out[0]["mem"] == 0.2
    assert out[1]["status"] == abi.CA_UTIL_NO_MEM
    assert out[8]["resource"] == abi.CA_UTIL_GPU and out[8]["gpu"] == 1.0
    info, err = U.info_from_row(out[1], "node1", None)
    assert err is not None and str(err) == "failed to get memory from node1" and info == U.Info()


def _empty_case():
    """cluster_test.go:39-70 (FindEmptyNodesToRemove): n1 empty; n2 runs an unreplicated
    pod (blocks); n3 a replicated pod (movable); n4 only a DaemonSet pod (empty)."""
    nodes = [build_test_node(f"n{i}", 1000, 2000000) for i in range(1, 5)]
    p2 = build_test_pod("p2", 300, 500000)
    p3 = set_rs_pod(build_test_pod("p3", 300, 500000), "rs")
    p4 = build_test_pod("p4", 300, 500000)
    p4.owner_refs = [OwnerReference("DaemonSet", "ds")]
    return [NodeInfo(nodes[0], []), NodeInfo(nodes[1], [p2]), NodeInfo(nodes[2], [p3]), NodeInfo(nodes[3], [p4])]


def test_oracle_empty_nodes(oracle_lib):
    nis = _empty_case()
    nodes, off, pods = U.build_table(nis, [None] * 4, NodeDeleteOptions(), 0.0)
    out = oracle_lib.node_utilization(nodes, off, pods, False, False, 0)
    assert [ni.node.name for ni, r in zip(nis, out) if r["empty"]] == ["n1", "n4"]


def test_oracle_random_edges(oracle_lib):
    """The generator's edge cases come out as the reference defines them."""
    nodes, off, pods, now = W.util_table(seed=3, n_nodes=2000, pods_per_node=10)
    out = oracle_lib.node_utilization(nodes, off, pods, True, True, now)
    st = out["status"]
    for code in (abi.CA_UTIL_NO_CPU, abi.CA_UTIL_ZERO_CPU, abi.CA_UTIL_NO_MEM, abi.CA_UTIL_ZERO_MEM):
        assert (st == code).any()
    assert np.isinf(out["utilization"]).any() or np.isnan(out["utilization"]).any()
    assert out["empty"].any() and not out["empty"].all()


# ---------------------------------------------------------------------------- GPU
def _bits_equal(a, b):
    return a.tobytes() == b.tobytes()


@pytest.mark.gpu
def test_gpu_info_test_cases(oracle_lib):
    from autoscaler_amd import native
    cases = info_test_cases()
    nodes, off, pods = _table(cases)
    t = native.UtilTable(0, nodes, off, pods)
    for sds in (False, True):
        for smp in (False, True):
            got = t.calculate(sds, smp, round(TEST_TIME * 1e9))
            ref = oracle_lib.node_utilization(nodes, off, pods, sds, smp, round(TEST_TIME * 1e9))
            assert _bits_equal(got, ref), (sds, smp)
    for i, (name, _, sds, smp, expected) in enumerate(cases):
        _check_expected(name, t.calculate(sds, smp, round(TEST_TIME * 1e9))[i], expected)
    t.close()


@pytest.mark.gpu
def test_gpu_api_calculate_and_empty():
    cases = info_test_cases()
    for name, ni, sds, smp, expected in cases:
        info, err = U.Calculate(ni, sds, smp, gpu_config_from_node(ni.node), TEST_TIME)
        if expected == "error":
            assert err is not None, name
        else:
            assert err is None and abs(info.Utilization - expected) <= 0.01 * max(expected, 1e-9), name
    assert U.FindEmptyNodesToRemove(_empty_case(), NodeDeleteOptions(), 0.0) == ["n1", "n4"]
    assert U.FindEmptyNodesToRemove([], NodeDeleteOptions(), 0.0) == []


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n_nodes,ppn", [(1, 1, 0), (2, 63, 3), (3, 2000, 10), (4, 5000, 30), (5, 777, 90),
                                              (6, 15000, 20)])
def test_gpu_random_parity(seed, n_nodes, ppn, oracle_lib):
    from autoscaler_amd import native
    nodes, off, pods, now = W.util_table(seed=seed, n_nodes=n_nodes, pods_per_node=ppn)
    t = native.UtilTable(0, nodes, off, pods)
    for sds, smp in ((False, False), (True, False), (True, True)):
        got = t.calculate(sds, smp, now)
        ref = oracle_lib.node_utilization(nodes, off, pods, sds, smp, now)
        assert _bits_equal(got, ref), (seed, sds, smp, np.nonzero(got != ref)[0][:8])
    t.close()


@pytest.mark.gpu
def test_gpu_empty_table():
    from autoscaler_amd import native
    t = native.UtilTable(0, np.zeros(0, abi.UTIL_NODE_DTYPE), np.zeros(1, np.int32), np.zeros(0, abi.UTIL_POD_DTYPE))
    assert len(t.calculate(True, True, 0)) == 0
    t.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n_nodes,ppn,n_add", [(7, 63, 3, 40), (8, 3000, 12, 5000), (9, 15000, 20, 17000)])
def test_gpu_added_pods_zero_copy(seed, n_nodes, ppn, n_add, oracle_lib):
    """ca_util_table_set_added (rows appended per node) with page-locked results written by
    the kernel (zero-copy) == the oracle over the merged table; set_added twice in a row
    (the staging buffer reused while the previous copy may be in flight) keeps the last."""
    from autoscaler_amd import native
    nodes, off, pods, now = W.util_table(seed=seed, n_nodes=n_nodes, pods_per_node=ppn)
    rng = np.random.default_rng(seed)
    add_node = rng.integers(0, n_nodes, n_add).astype(np.int32)
    add = pods[rng.integers(0, len(pods), n_add)] if len(pods) else np.zeros(n_add, abi.UTIL_POD_DTYPE)
    # the merged reference table: each node's rows, then its added pods in call order
    node_of = np.concatenate([np.repeat(np.arange(n_nodes), np.diff(off)), add_node])
    order = np.argsort(node_of, kind="stable")
    m_pods = np.concatenate([pods, add])[order]
    m_off = np.zeros(n_nodes + 1, np.int32)
    np.cumsum(np.bincount(node_of, minlength=n_nodes), out=m_off[1:])
    t = native.UtilTable(0, nodes, off, pods)
    rows = native.PinnedRows()
    t.set_added(add_node[::-1].copy(), add[::-1].copy())          # replaced by the next call
    t.set_added(add_node, add)
    for sds, smp in ((False, False), (True, True)):
        out = rows.zeros("info", n_nodes, abi.UTIL_INFO_DTYPE)
        got = t.calculate(sds, smp, now, out=out)
        ref = oracle_lib.node_utilization(nodes, m_off, m_pods, sds, smp, now)
        assert _bits_equal(got, ref), (seed, sds, smp)
        assert _bits_equal(t.calculate(sds, smp, now), ref)       # pageable: the DMA path
    # page-locked added arrays (copied in place), then an update: the per-node sums of the
    # added pods are consumed by every calculate and nothing of them survives an update
    pn = rows.zeros("add_node", n_add, np.int32)
    pp = rows.zeros("add_pods", n_add, abi.UTIL_POD_DTYPE)
    pn[:] = add_node
    pp[:] = add
    t.set_added(pn, pp)
    out = rows.zeros("info", n_nodes, abi.UTIL_INFO_DTYPE)
    assert _bits_equal(t.calculate(True, False, now, out=out), oracle_lib.node_utilization(nodes, m_off, m_pods, True,
                                                                                            False, now))
    t.update(nodes, off, pods)
    assert _bits_equal(t.calculate(False, False, now), oracle_lib.node_utilization(nodes, off, pods, False, False, now))
    t.close()
    rows.close()
