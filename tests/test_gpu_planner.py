"""GPU parity of the planner's committing removal loop (ca_plan_removals)
against the oracle (or_plan_removals, itself checked against a step-by-step restatement
in tests/test_planner.py and the reference's planner_test.go in the golden cases):
bit-exact results, moves, hints, lastIndex, PDB budgets, and the committed snapshot.

Both device paths run every case: the device-resident chain (plan_chain.hip, the default
where it applies) and the speculative sweep windows (CASIM_PLAN_SPECULATIVE, and the
fallback for pods with host ports / extended resources or rows beyond LDS)."""
from __future__ import annotations

import numpy as np
import pytest

from autoscaler_amd import abi, native
from autoscaler_amd import workloads as W
from conftest import gpu_available
from plangen import PlanCase, rand_plan_case

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="no HIP device")]


@pytest.fixture(scope="module")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle


_M = {}


def _mirror():
    if "m" not in _M:
        _M["m"] = native.Mirror(0)
    m = _M["m"]
    m.clear()
    return m


def _check(o, g, what=""):
    assert np.array_equal(o.results, g.results), (what, o.results, g.results)
    assert np.array_equal(o.moves, g.moves), what
    assert np.array_equal(o.hints, g.hints), what
    assert o.last_index == g.last_index, what
    assert np.array_equal(o.allowed, g.allowed), what


def _follow_up_sweep(b, n_nodes: int, n_pods: int):
    """A legacy FindNodesToRemove over every node of the committed snapshot: equal outputs
    on both backends mean equal committed rows and pod lists."""
    cands = np.arange(n_nodes, dtype=np.int32)
    off, moves = [0], []
    for c in range(n_nodes):
        moves.extend(b.node_pods(c))
        off.append(len(moves))
    return b.find_nodes_to_remove(cands, np.ones(n_nodes, np.uint8), np.zeros(n_nodes, np.int32),
                                  np.array(off, np.int32), np.array(moves, np.int32),
                                  np.full(n_pods, -1, np.int32), 0)


@pytest.fixture(params=["chain", "chain1", "speculative"])
def path(request, monkeypatch):
    """The device chain with its helper waves (default), the chain alone (one wavefront:
    CASIM_PLAN_HELPERS=0), and the speculative sweep windows."""
    if request.param == "speculative":
        monkeypatch.setenv("CASIM_PLAN_SPECULATIVE", "1")
    else:
        monkeypatch.delenv("CASIM_PLAN_SPECULATIVE", raising=False)
        monkeypatch.setenv("CASIM_PLAN_HELPERS", "0" if request.param == "chain1" else "7")
    return "chain" if request.param.startswith("chain") else request.param


def _no_ext(case: PlanCase) -> PlanCase:
    """The case without host ports and extended-resource requests (the chain's scope)."""
    p = case.table.pods
    p["port_conflict"] = 0
    p["port_use"] = 0
    p["req_scalar"] = 0
    p["tpu_scalar_mask"] = 0
    p["flags"] &= ~np.uint32(abi.CA_POD_HAS_SCALAR_KEYS | abi.CA_POD_HAS_NONTPU_SCALAR_KEYS)
    return case


def _run_both(case: PlanCase, oracle):
    outs = []
    for b in (oracle.OracleState(), _mirror()):
        case.load(b)
        out = case.plan(b)
        n_nodes = len(case.node_recs)
        n_pods = len(case.table) + len(out.moves)
        outs.append((out, [b.node_pods(i) for i in range(n_nodes)], _follow_up_sweep(b, n_nodes, n_pods)))
    (o, on, os_), (g, gn, gs) = outs
    _check(o, g)
    assert on == gn
    assert np.array_equal(os_.results, gs.results) and np.array_equal(os_.dest, gs.dest)
    return o, g


@pytest.mark.parametrize("seed", range(40))
def test_plan_random(seed, oracle, path):
    case = rand_plan_case(seed, n_nodes=10 + seed % 7, pods_per_node=3 + seed % 3, n_pdbs=(seed % 3) * 2)
    _run_both(case, oracle)


@pytest.mark.parametrize("seed", range(40))
def test_plan_random_chain_scope(seed, oracle):
    """The random cases without ports / extended resources run on the device chain."""
    case = _no_ext(rand_plan_case(seed, n_nodes=10 + seed % 7, pods_per_node=3 + seed % 3, n_pdbs=(seed % 3) * 2))
    _run_both(case, oracle)
    assert _M["m"].plan_stats()["path"] == "chain"


@pytest.mark.parametrize("seed", range(8))
def test_plan_random_larger(seed, oracle, path):
    """More candidates per window: commits inside a speculation window conflict with later
    speculations (placements on filled nodes, hints on removed nodes, grown pod lists)."""
    case = rand_plan_case(100 + seed, n_nodes=60, pods_per_node=6, n_pdbs=3, limit=0)
    _run_both(case, oracle)


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("help_after", ["1", "2"])
def test_plan_random_larger_chain_scope_helpers(seed, help_after, oracle, monkeypatch):
    """The helper waves take every scan after its first (help_after = 1) or second block:
    same results as the oracle (blocks scanned out of order, maxima refreshed by helpers)."""
    monkeypatch.setenv("CASIM_PLAN_HELPERS", "7")
    monkeypatch.setenv("CASIM_PLAN_HELP_AFTER", help_after)
    case = _no_ext(rand_plan_case(200 + seed, n_nodes=150 + 61 * seed, pods_per_node=6, n_pdbs=3, limit=0))
    _run_both(case, oracle)
    assert _M["m"].plan_stats()["path"] == "chain"


@pytest.mark.parametrize("seed", range(8))
def test_plan_random_larger_chain_scope(seed, oracle):
    """Copies moved again (committed onto a later candidate), PDB budgets running out,
    hints to removed nodes, ragged 1-block rings — on the device chain."""
    case = _no_ext(rand_plan_case(100 + seed, n_nodes=60 + 13 * seed, pods_per_node=6, n_pdbs=3, limit=0))
    _run_both(case, oracle)
    assert _M["m"].plan_stats()["path"] == "chain"


def test_plan_fork_revert(oracle, path):
    """UpdateClusterState forks around the loop (planner.go:108-110): after Revert the mirror
    is the snapshot it was, and simulates as the oracle's reverted one does."""
    case = rand_plan_case(7, n_nodes=30, pods_per_node=5, limit=0)
    o, m = oracle.OracleState(), _mirror()
    for b in (o, m):
        case.load(b)
        b.fork()
    po, pm = case.plan(o), case.plan(m)
    _check(po, pm)
    assert len(pm.moves) > 0
    for b in (o, m):
        b.revert()
    n = len(case.node_recs)
    assert [o.node_pods(i) for i in range(n)] == [m.node_pods(i) for i in range(n)]
    assert [m.node_pods(i) for i in range(n)] == [
        [int(j) for j in np.nonzero(case.node_of == i)[0]] for i in range(n)]
    so = _follow_up_sweep(o, n, len(case.table) + len(po.moves))
    sm = _follow_up_sweep(m, n, len(case.table) + len(pm.moves))
    assert np.array_equal(so.results, sm.results) and np.array_equal(so.dest, sm.dest)


def _c3_case(n_nodes: int, limit: int, hints=None) -> PlanCase:
    w = W.c3(n_nodes=n_nodes)
    return PlanCase(w.nodes, w.table, w.pod_node, w.candidates, w.dest_mask, w.cand_status, w.move_off,
                    w.move_pods, np.full(len(w.table), -1, np.int32) if hints is None else hints, 0, limit,
                    np.zeros(0, np.int32), np.zeros(1, np.int32), np.zeros(0, np.int32))


@pytest.mark.parametrize("n_nodes,limit", [(1500, 0), (5000, 20), (5000, 200), (5000, 0)])
def test_plan_c3(n_nodes, limit, oracle, path):
    """(5000, 0), speculative: the late windows over a nearly full cluster go through the
    sweep's serial exact chain and serial-only calls."""
    case = _c3_case(n_nodes, limit)
    o, m = oracle.OracleState(), _mirror()
    case.load(o)
    case.load(m)
    po, pm = case.plan(o), case.plan(m)
    _check(po, pm, f"C3 n={n_nodes} limit={limit}")
    removed = int(po.results["removable"].sum())
    assert removed == limit if limit else removed > 0
    st = m.plan_stats()
    assert st["rounds"] >= 1 and st["simulated"] >= 1
    assert st["path"] == path


def test_plan_c4_attributes(oracle, path):
    """Taints, labels, selectors and required terms on the C4 sweep workload."""
    w = W.c4_sweep(n_nodes=800)
    case = PlanCase(w.nodes, w.table, w.pod_node, w.candidates, w.dest_mask, w.cand_status, w.move_off,
                    w.move_pods, np.full(len(w.table), -1, np.int32), 3, 0, np.zeros(0, np.int32),
                    np.zeros(1, np.int32), np.zeros(0, np.int32))
    o, m = oracle.OracleState(), _mirror()
    W.load_sweep(o, w)
    W.load_sweep(m, w)
    _check(case.plan(o), case.plan(m), "C4")


@pytest.mark.parametrize("which", ["chain", "speculative"])
def test_plan_failure_is_atomic(oracle, monkeypatch, which):
    """an error in a later speculation round (injected: CASIM_PLAN_FAIL_ROUND=3),
    or after the device chain replayed its commits into the mirror (CASIM_PLAN_FAIL_ROUND=1),
    leaves nothing of the call behind — mirror rows and pod lists, PDB budgets, hints,
    lastIndex — and the same call then succeeds exactly like the oracle's."""
    case = rand_plan_case(101, n_nodes=60, pods_per_node=6, n_pdbs=3, limit=0)
    if which == "chain":
        _no_ext(case)
    m = _mirror()
    case.load(m)
    n = len(case.node_recs)
    before = [m.node_pods(i) for i in range(n)]
    if which == "speculative":
        monkeypatch.setenv("CASIM_PLAN_SPECULATIVE", "1")
        monkeypatch.setenv("CASIM_PLAN_WINDOW", "8")          # several rounds, commits in each
    monkeypatch.setenv("CASIM_PLAN_FAIL_ROUND", "3" if which == "speculative" else "1")
    with pytest.raises(native.CasimError):
        case.plan(m)
    monkeypatch.delenv("CASIM_PLAN_FAIL_ROUND")
    assert [m.node_pods(i) for i in range(n)] == before
    g = case.plan(m)
    o_b = oracle.OracleState()
    case2 = rand_plan_case(101, n_nodes=60, pods_per_node=6, n_pdbs=3, limit=0)
    if which == "chain":
        _no_ext(case2)
    case2.load(o_b)
    o = case2.plan(o_b)
    # the copies' pod ids: records stored by the failed call are detached, never reused
    shift = int(g.moves["new_pod"].min()) - int(o.moves["new_pod"].min())
    assert shift >= 0 and np.array_equal(o.moves["new_pod"] + shift, g.moves["new_pod"])
    g.moves["new_pod"] -= shift
    _check(o, g, "after an injected failure")
    st = m.plan_stats()
    assert st["path"] == which
    assert st["rounds"] >= (2 if which == "speculative" else 1)
