"""Multi-device entry points of the C ABI (multi.hip, casim.h "multi-GPU"): node groups /
sweep candidates in contiguous blocks over replicated mirrors, run concurrently from the
caller's lastIndex, chain fixed up inside the library.  The box has one GPU, so the
replicas are several mirrors on device 0 — the blocks, threads, re-runs and re-basing are
the same code as on 8 GPUs.  Results must equal one mirror's call and the oracle, bit for
bit (the blocks are coupled only through lastIndex)."""
import dataclasses

import numpy as np
import pytest

from autoscaler_amd import native
from autoscaler_amd import workloads as W
from estgen import _encode_estimate, _estimate_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle


def _replicas(n, load):
    ms = [native.Mirror(0) for _ in range(n)]
    for m in ms:
        load(m)
    return ms


def _eq_estimate(ro, g, off):
    assert np.array_equal(ro.results, g.results)
    assert ro.last_index == g.last_index
    for k in range(len(off) - 1):
        if int(ro.results[k]["status"]) != 0:
            continue
        a, n = off[k], int(ro.results[k]["n_scheduled"])
        assert np.array_equal(ro.sched_pod[a:a + n], g.sched_pod[a:a + n]), k
        assert np.array_equal(ro.sched_node[a:a + n], g.sched_node[a:a + n]), k


@pytest.mark.parametrize("replicas", [2, 3, 5])
@pytest.mark.parametrize("seed", range(6))
def test_multi_estimate_random(seed, replicas, oracle):
    """Random clusters (existing nodes, ports, taints, scalars): the blocks' lastIndex
    dependence varies, so re-runs and re-basing both occur across the seeds."""
    rng, nodes, pods, templates, groups = _estimate_inputs(seed, n_groups=9, n_pods=70)
    table, node_recs, tm, off, pod_idx = _encode_estimate(nodes, pods, templates, groups)
    max_nodes = [0, 1, 3, 40][seed % 4]
    L0 = [0, 3, 11][seed % 3]
    o = oracle.OracleState()
    o.clear()
    if len(node_recs):
        o.add_nodes(node_recs)
    ro = o.estimate(table, off, pod_idx, tm, max_nodes, L0)

    def load(m):
        if len(node_recs):
            m.add_nodes(node_recs)
    ms = _replicas(replicas, load)
    with native.Multi(ms) as mm, native.MultiEstimatePlan(mm, table, off, pod_idx, tm) as plan:
        for _ in range(2):
            g = plan.run(max_nodes, L0)
            _eq_estimate(ro, g, off)
        st = plan.stats()
        assert st["blocks"] == min(replicas, len(tm))
    for m in ms:
        m.close()


def test_multi_estimate_c2(oracle):
    """C2-shaped batch over 4 replicas vs one mirror (the bench's strong-scaling split)."""
    w = W.c2(n_pods=12000, n_groups=24, n_existing=200)
    single = native.Mirror(0)
    W.load_estimate(single, w)
    ref = single.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 5)
    ms = _replicas(4, lambda m: W.load_estimate(m, w))
    with native.Multi(ms) as mm, native.MultiEstimatePlan(mm, w.table, w.group_off, w.pod_idx, w.templates) as plan:
        g = plan.run(w.max_nodes, 5)
        _eq_estimate(ref, g, w.group_off)
        assert plan.stats()["blocks"] == 4
    for m in ms + [single]:
        m.close()


@pytest.mark.parametrize("compose", ["map", "serial"])
@pytest.mark.parametrize("replicas", [2, 4])
@pytest.mark.parametrize("n_nodes", [300, 1500])
def test_multi_sweep(n_nodes, replicas, compose, oracle, monkeypatch):
    """C3 sweep with fresh hints (every candidate's scans succeed: every block depends on
    its input lastIndex), then the second loop with the first loop's hints (hint
    placements: blocks pass lastIndex through).  'map': the blocks' lastIndex classes are
    composed on the host and every block resolves from its exact input at once;
    'serial' (CASIM_MULTI_NO_MAP): blocks run from the caller's input, later ones re-run."""
    if compose == "serial":
        monkeypatch.setenv("CASIM_MULTI_NO_MAP", "1")
    w = W.c3(n_nodes=n_nodes)
    args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
    o = oracle.OracleState()
    W.load_sweep(o, w)
    o1 = o.find_nodes_to_remove(*args, np.full(len(w.table), -1, np.int32), 7)
    o2 = o.find_nodes_to_remove(*args, o1.hints, o1.last_index)
    ms = _replicas(replicas, lambda m: W.load_sweep(m, w))
    with native.Multi(ms) as mm, native.MultiRemovalPlan(mm, *args) as plan:
        g1 = plan.run(np.full(len(w.table), -1, np.int32), 7)
        assert np.array_equal(o1.results, g1.results) and o1.last_index == g1.last_index
        assert np.array_equal(o1.dest, g1.dest) and np.array_equal(o1.hints, g1.hints)
        s1 = plan.stats()
        assert s1["blocks"] == replicas
        if compose == "serial":
            assert s1["reruns"] >= 1
        g2 = plan.run(g1.hints, g1.last_index)
        assert np.array_equal(o2.results, g2.results) and o2.last_index == g2.last_index
        assert np.array_equal(o2.dest, g2.dest) and np.array_equal(o2.hints, g2.hints)
    for m in ms:
        m.close()


def test_multi_sweep_prefix_protocol(oracle):
    """An out-of-scope pod to move in a middle block: that candidate reports
    OUT_OF_SCOPE, every later candidate (later blocks included) NOT_RUN."""
    from autoscaler_amd import abi
    w = W.c3(n_nodes=300)
    table = w.table
    pods = table.pods.copy()
    c_mid = len(w.candidates) * 2 // 3
    victim = int(w.move_pods[w.move_off[c_mid]])
    pods["flags"][victim] |= abi.CA_POD_OUT_OF_SCOPE
    w2 = dataclasses.replace(w, table=abi.PodTable(pods))
    args = (w2.candidates, w2.dest_mask, w2.cand_status, w2.move_off, w2.move_pods)
    single = native.Mirror(0)
    W.load_sweep(single, w2)
    ref = single.find_nodes_to_remove(*args, np.full(len(w2.table), -1, np.int32), 0)
    ms = _replicas(3, lambda m: W.load_sweep(m, w2))
    with native.Multi(ms) as mm, native.MultiRemovalPlan(mm, *args) as plan:
        g = plan.run(np.full(len(w2.table), -1, np.int32), 0)
    assert np.array_equal(ref.results, g.results) and ref.last_index == g.last_index
    assert int(g.results[c_mid]["reason"]) == abi.CA_UNREMOVABLE_OUT_OF_SCOPE
    assert (g.results["reason"][c_mid + 1:] == abi.CA_UNREMOVABLE_NOT_RUN).all()
    for m in ms + [single]:
        m.close()


@pytest.mark.parametrize("replicas", [2, 4])
def test_multi_sweep_c3_full(replicas, oracle):
    """BASELINE C3 at full size (5k nodes, 150k pods) on ca_multi_*: the fresh loop (every
    block lastIndex-sensitive in a loose cluster: the blocks' lastIndex maps compose on the
    host, so none waits for its predecessor or runs twice) and the hinted second loop (hint
    placements pass lastIndex through), against the oracle, with no re-run candidates."""
    w = W.c3()
    args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
    o = oracle.OracleState()
    W.load_sweep(o, w)
    o1 = o.find_nodes_to_remove(*args, np.full(len(w.table), -1, np.int32), 0)
    o2 = o.find_nodes_to_remove(*args, o1.hints, o1.last_index)
    ms = _replicas(replicas, lambda m: W.load_sweep(m, w))
    with native.Multi(ms) as mm, native.MultiRemovalPlan(mm, *args) as plan:
        g1 = plan.run(np.full(len(w.table), -1, np.int32), 0)
        assert np.array_equal(o1.results, g1.results) and o1.last_index == g1.last_index
        assert np.array_equal(o1.dest, g1.dest) and np.array_equal(o1.hints, g1.hints)
        s1 = plan.stats()
        print(f"C3 fresh, {replicas} blocks: re-run blocks {s1['reruns']}, candidates {s1['rerun_candidates']}")
        # the blocks' lastIndex maps compose from the true input: no block waits for its
        # predecessor and none runs twice
        assert s1["rerun_candidates"] == 0
        g2 = plan.run(g1.hints, g1.last_index)
        assert np.array_equal(o2.results, g2.results) and o2.last_index == g2.last_index
        assert np.array_equal(o2.dest, g2.dest) and np.array_equal(o2.hints, g2.hints)
        s2 = plan.stats()
        print(f"C3 hinted, {replicas} blocks: re-run blocks {s2['reruns']}, candidates {s2['rerun_candidates']}")
        assert s2["rerun_candidates"] == 0
    for m in ms:
        m.close()


def test_multi_estimate_c4_full(oracle):
    """BASELINE C4 at full size (50k pods x 100 groups, taints / node affinity) on
    ca_multi_estimate_plan over 2 replicas: identical to one mirror and the Go-order
    oracle; the re-run groups are reported."""
    w = W.c4()
    o = oracle.OracleState()
    W.load_estimate(o, w)
    ro = o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 0)
    ms = _replicas(2, lambda m: W.load_estimate(m, w))
    with native.Multi(ms) as mm, native.MultiEstimatePlan(mm, w.table, w.group_off, w.pod_idx, w.templates) as plan:
        g = plan.run(w.max_nodes, 0)
        _eq_estimate(ro, g, w.group_off)
        st = plan.stats()
        print(f"C4, 2 blocks: re-run blocks {st['reruns']}, groups {st['rerun_groups']}")
        assert st["blocks"] == 2
    for m in ms:
        m.close()


def test_multi_sweep_loops_reuse_plan(oracle):
    """a range whose probe makes no successful scan but has sensitive candidates
    must build this call's tables before it resolves (never walk an earlier call's).  One
    plan on 4 replicas of a 300-node C3, loops in the order fresh, hinted, fresh from another
    input, hinted again, and a second plan whose very first call is the hinted loop: every
    call against the oracle."""
    w = W.c3(n_nodes=300)
    args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
    o = oracle.OracleState()
    W.load_sweep(o, w)
    fresh = np.full(len(w.table), -1, np.int32)
    o1 = o.find_nodes_to_remove(*args, fresh, 7)
    o2 = o.find_nodes_to_remove(*args, o1.hints, o1.last_index)
    o3 = o.find_nodes_to_remove(*args, fresh, 123)
    o4 = o.find_nodes_to_remove(*args, o1.hints, 45)
    seq = [(fresh, 7, o1), (o1.hints, o1.last_index, o2), (fresh, 123, o3), (o1.hints, 45, o4), (o1.hints, 45, o4)]
    ms = _replicas(4, lambda m: W.load_sweep(m, w))
    with native.Multi(ms) as mm:
        with native.MultiRemovalPlan(mm, *args) as plan:
            for h, L, ro in seq:
                g = plan.run(h.copy(), L)
                assert np.array_equal(ro.results, g.results) and ro.last_index == g.last_index
                assert np.array_equal(ro.dest, g.dest) and np.array_equal(ro.hints, g.hints)
        with native.MultiRemovalPlan(mm, *args) as plan:           # first call: the hinted loop
            for h, L, ro in seq[3:] + seq[:2]:
                g = plan.run(h.copy(), L)
                assert np.array_equal(ro.results, g.results) and ro.last_index == g.last_index
                assert np.array_equal(ro.dest, g.dest) and np.array_equal(ro.hints, g.hints)
    for m in ms:
        m.close()


@pytest.mark.parametrize("what", ["estimate", "sweep"])
def test_multi_distinct_devices(what, oracle):
    """Replicas on distinct devices (one per GPU): per-thread device binding, each device's
    zero-copy publisher writing its slice of one page-locked buffer, events and streams per
    device.  Same outputs as the oracle.  Skipped on a one-GPU box."""
    if native.device_count() < 2:
        pytest.skip("needs two or more GPUs: replicas on distinct devices")
    D = min(native.device_count(), 4)
    if what == "estimate":
        w = W.c2(n_pods=6000, n_groups=16, n_existing=100)
        o = oracle.OracleState()
        W.load_estimate(o, w)
        ro = o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 3)
        ms = [native.Mirror(d) for d in range(D)]
        for m in ms:
            W.load_estimate(m, w)
        with native.Multi(ms) as mm, native.MultiEstimatePlan(mm, w.table, w.group_off, w.pod_idx, w.templates) as plan:
            for _ in range(2):
                g = plan.run(w.max_nodes, 3)
                _eq_estimate(ro, g, w.group_off)
    else:
        w = W.c3(n_nodes=1500)
        args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
        o = oracle.OracleState()
        W.load_sweep(o, w)
        o1 = o.find_nodes_to_remove(*args, np.full(len(w.table), -1, np.int32), 0)
        ms = [native.Mirror(d) for d in range(D)]
        for m in ms:
            W.load_sweep(m, w)
        with native.Multi(ms) as mm, native.MultiRemovalPlan(mm, *args) as plan:
            g = plan.run(np.full(len(w.table), -1, np.int32), 0)
            assert np.array_equal(o1.results, g.results) and o1.last_index == g.last_index
            assert np.array_equal(o1.dest, g.dest) and np.array_equal(o1.hints, g.hints)
    for m in ms:
        m.close()
